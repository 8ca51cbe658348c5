// ksim_pgen.h — host/device interface of the general persistent kernel (ksim_pgen.hip): pods with
// inter-pod affinity, SelectorSpread, volumes or CheckServiceAffinity in one launch per call.
#pragma once
#include "ksim_common.h"

// ---- per-pod context record (built by ksim_pgen_pack before the launch, one per queued pod) ----
// Everything the per-pod cycle reads besides the node rows, denormalised from the class, affinity
// and volume tables into one contiguous record, so the kernel stages pod p+1's record into LDS
// with a handful of independent loads while pod p's exchange is in flight.
//   [ksim_pod 128 B][PgHdr 64 B][tv 16 x i64][av 16 x i64][ad 16 x i64]   = PG_REC_FIXED bytes
//   then 16-byte aligned sections (counts in the header):
//   anti  i32 [n_anti]   carried required anti-affinity terms the pod's identity matches
//   prio  i32 [n_prio]   carried priority terms the identity matches
//   req   i32x4 [n_req]  own required terms: pair, gate key, exist pair, kind | self_ok << 8
//   pref  {i32 pair, i32 pad, i64 weight} [n_pref]  own preferred terms
//   mp    i32x2 [n_mp]   counted pairs the identity matches: pair, key        (commit)
//   car   {i32 term, i32 key, i64 amount} [n_car]   carried amounts the pod brings (commit)
//   ref   i32x4 [n_ref]  volume refs: key, flags, key_filter, pad
//   zok   u32 [n_zw]     NoVolumeZoneConflict verdict bits of the pod's volume class per label set
//   port  u64 [n_port]   host-port keys
//   scal  ksim_scalar_req [n_scal]
#define PG_REC_FIXED (128 + 64 + 3 * KSIM_MAX_RCLASS * 8)
#define PG_REC_MAX 6144

// header flags
#define PGF_AFF 1     // the pod takes part in inter-pod affinity (identity or class)
#define PGF_IPA 2     // reads the InterPodAffinity priority (pass A min / max)
#define PGF_SHARED 4  // its commit changes counts in a topology domain several nodes share
#define PGF_VOL 8     // has a volume class
#define PGF_NOHYP 16  // its commit leaves the rows' LDS image (gpu / ephemeral / scalar requests, shared domains)
#define PGF_AUX 32    // reads the auxiliary priority (ksim_affinity_tables.aux_*); its counted pair + 1 in
                      // bits 8.. (0: none — serviceAntiAffinity still scores by the row's label)
#define PGF_AUX_SHIFT 8

struct PgHdr {
  int32_t K, k1, k2, sp;  // reduce classes (K = k1 * k2), SelectorSpread pair or -1
  int32_t fl;             // PGF_*
  int32_t n_anti, n_req, n_pref;
  int32_t n_prio, n_mp, n_car, n_ref;
  int32_t vfilter, n_zw, n_port, n_scal;
};
static_assert(sizeof(PgHdr) == 64, "PgHdr is 64 bytes");

enum { PGS_ANTI, PGS_PRIO, PGS_REQ, PGS_PREF, PGS_MP, PGS_CAR, PGS_REF, PGS_ZOK, PGS_PORT, PGS_SCAL, PGS_END };

// byte offsets of the record's sections from its header counts
__host__ __device__ inline void pg_sections(const PgHdr& h, uint32_t* off) {
  auto a16 = [](uint32_t b) { return (b + 15u) & ~15u; };
  uint32_t o = PG_REC_FIXED;
  off[PGS_ANTI] = o; o += a16(4u * h.n_anti);
  off[PGS_PRIO] = o; o += a16(4u * h.n_prio);
  off[PGS_REQ] = o;  o += 16u * h.n_req;
  off[PGS_PREF] = o; o += 16u * h.n_pref;
  off[PGS_MP] = o;   o += a16(8u * h.n_mp);
  off[PGS_CAR] = o;  o += 16u * h.n_car;
  off[PGS_REF] = o;  o += 16u * h.n_ref;
  off[PGS_ZOK] = o;  o += a16(4u * h.n_zw);
  off[PGS_PORT] = o; o += a16(8u * h.n_port);
  off[PGS_SCAL] = o; o += a16(24u * h.n_scal);
  off[PGS_END] = o;
}

// ---- LDS image of a workgroup (offsets planned on the host by ksim_pgen_plan) ----
enum {
  PGO_AC, PGO_AM, PGO_RC, PGO_RM, PGO_ZC, PGO_ZM,  // i64 [chunk]: the 60-byte resource row
  PGO_AL, PGO_CT, PGO_FL, PGO_LS, PGO_TS,          // i32 [chunk]
  PGO_SC,                                          // i32 [chunk] this pod's score (-1: does not fit)
  PGO_CL,                                          // u8  [chunk] its reduce class
  PGO_ST,                                          // u16 [n_st][chunk] static (pod class, row) words
  PGO_VC,                                          // i32 [chunk] volume slots used
  PGO_VH,                                          // u16 [3][chunk] mounted keys per MaxPD filter
  PGO_VS,                                          // u64 [vslots][chunk] volume slots
  PGO_PC,                                          // i32 [chunk] host-port slots used
  PGO_PK,                                          // u64 [pslots][chunk] host-port keys
  PGO_DOM,                                         // i32 [n_keys][chunk] topology domains
  PGO_CNT,                                         // i32 [n_pair][chunk] counted pairs, row form
  PGO_CAR,                                         // i64 [n_carry][chunk] carried terms, row form
  PGO_X0, PGO_X1, PGO_X2, PGO_X3,                  // four pod-context records (ring)
  PGO_E1,                                          // PgEv [chunk] the rows' E1 evaluations (dual form)
  PGO_HD, PGO_HC, PGO_HK,                          // dense hypothesis deltas (dual form, when they fit):
                                                   //   i32 [n_pair] key + 1 of pod p's count on pair c,
                                                   //   i64 [n_carry] its carried amount of term e, i32 key + 1
  PGO_N
};

struct PgDims {
  int32_t n_st;     // pod classes whose static words are staged (0: computed from the tables)
  int32_t vcap;     // volume slots per node in the tables (0: no volume tables)
  int32_t vslots;   // of which the first vslots (<= PG_VS_LDS) are staged in LDS, the rest stay in HBM
  int32_t pslots;   // host-port slots per row (0: none)
  int32_t n_keys, n_pair, n_carry;
  int32_t rec_stride;
  int32_t hyp;      // 1: the dual-hypothesis kernel's layout (PGO_E1 and four records)
  int32_t hdense;   // 1: the dense hypothesis deltas are staged (PGO_HD / HC / HK)
};
#define PG_VS_LDS 8
#define PG_EV_BYTES 40  // sizeof(PgEv) (ksim_pgen.hip)

// Arguments beyond the context.  The affinity / volume descriptors travel by value (kernel
// arguments stay in scalar registers instead of being re-read from HBM after every barrier).
struct PGenArgs {
  uint64_t* gran;     // exchange: pass-A records, class granules, commit words (PG_* in ksim_pgen.hip)
  char* rec;          // [count][rec_stride] pod-context records of the call
  const uint8_t* ident_shared;   // [n_ident] the identity's counted pairs include a shared-domain key
  const uint8_t* aclass_shared;  // [n_aclass] the class carries a term on a shared-domain key
  // identity lists (CSR, built by ksim_load_affinity): carried anti / priority terms it matches,
  // counted pairs it matches (pair, key)
  const int32_t* id_anti_off; const int32_t* id_anti;
  const int32_t* id_prio_off; const int32_t* id_prio;
  const int32_t* id_mp_off; const int32_t* id_mp;
  KsimAff A;          // valid when has_aff
  KsimVol V;          // valid when has_vol
  PgDims d;
  uint32_t off[PGO_N];
  int32_t has_aff, has_vol;
  int32_t n_zone;     // zones of the spread reduce (<= PG_MAXZ)
  int32_t svc_on;     // CheckServiceAffinity's lender check (A.svc_*; single-hypothesis kernel, n_pair <= PG_SVC_PAIRS)
  uint64_t spin_ticks;
  int32_t test_stall;  // diagnostic (KSIM_PGEN_TEST_STALL): the last workgroup exits at once, as one
                       // that never became resident; the others must abort and the host recover
};

extern "C" hipError_t ksim_launch_pgen2(const KsimCtx* c, const PGenArgs* g, int grid, int npt, size_t lds, hipStream_t s);
extern "C" hipError_t ksim_launch_pgen(const KsimCtx* c, const PGenArgs* g, int grid, int npt, size_t lds, hipStream_t s);
extern "C" hipError_t ksim_pgen_pack(const KsimCtx* c, const PGenArgs* g, hipStream_t s);
// LDS plan for `chunk` rows per workgroup: fills off[], returns the dynamic LDS bytes.
extern "C" size_t ksim_pgen_plan(int64_t chunk, const PgDims* d, uint32_t* off);
extern "C" size_t ksim_pgen_lds_budget(void);
extern "C" size_t ksim_pgen_gran_bytes(void);
extern "C" int ksim_pgen_max_zones(void);
extern "C" int ksim_pgen_max_aux_domains(void);
#define PG_SVC_PAIRS 256  // counted pairs whose domain-0 counts a workgroup keeps (the lender check's totals)
