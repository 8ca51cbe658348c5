// ksim_persistent.hip — persistent-kernel mode (placeholder until the persistent
// scheduler lands: reports "does not fit" so KSIM_MODE_AUTO uses launch mode).
#include "ksim_common.h"

extern "C" int ksim_persistent_config(int64_t n, int* grid, int* lds_rows) {
  (void)n;
  *grid = 0;
  *lds_rows = 0;
  return 0;
}

extern "C" hipError_t ksim_launch_persistent(const KsimCtx* c, int grid, int lds_rows, hipStream_t s) {
  (void)c; (void)grid; (void)lds_rows; (void)s;
  return hipErrorNotSupported;
}
