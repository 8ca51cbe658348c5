"""ctypes binding of libksim.so (include/ksim.h).  This is the only module that touches
the native library; it fails loudly when the library is missing — there is no CPU
fallback on the product path."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# KSIM_LIB selects another build of the same library (the diagnostic stamps build)
LIB_PATH = os.environ.get("KSIM_LIB") or os.path.join(PKG_DIR, "lib", "libksim.so")

KSIM_OK = 0
E_INVAL, E_DEVICE, E_NOMEM, E_UNSUPPORTED, E_STATE, E_OVERFLOW, E_NO_NODES = -1, -2, -3, -4, -5, -6, -7
ABI_VERSION = 7
MAX_SCALAR = 8
MAX_RCLASS = 16
MAX_WIDE = 256  # reduce classes per pod (KSIM_MAX_WIDE)
NREASONS = 32

# predicate bits
P_CHECK_NODE_CONDITION = 1 << 0
P_CHECK_NODE_UNSCHEDULABLE = 1 << 1
P_GENERAL = 1 << 2
P_HOSTNAME = 1 << 3
P_HOST_PORTS = 1 << 4
P_NODE_SELECTOR = 1 << 5
P_RESOURCES = 1 << 6
P_TAINTS = 1 << 7
P_NOEXEC_TAINTS = 1 << 8
P_MEM_PRESSURE = 1 << 9
P_DISK_PRESSURE = 1 << 10
P_LABEL_PRESENCE = 1 << 11
P_INTERPOD_AFFINITY = 1 << 12
P_DISK_CONFLICT = 1 << 13
P_MAX_EBS = 1 << 14
P_MAX_GCE_PD = 1 << 15
P_MAX_AZURE_DISK = 1 << 16
P_VOLUME_ZONE = 1 << 17
P_SERVICE_AFFINITY = 1 << 18

W_LEAST, W_MOST, W_BALANCED, W_TAINT_TOL, W_NODE_AFF, W_INTERPOD, W_SPREAD = range(7)
NW = 7

N_NOT_READY, N_OUT_OF_DISK, N_NET_UNAVAIL, N_UNSCHEDULABLE = 1, 2, 4, 8
N_MEM_PRESSURE, N_DISK_PRESSURE, N_LABEL_PRESENCE = 16, 32, 64

POD_ANY_REQUEST, POD_BEST_EFFORT, POD_NEED_SELECTOR, POD_NEED_TAINTS, POD_NEED_SVC_AFFINITY = 1, 2, 4, 8, 16

MODE_AUTO, MODE_LAUNCH, MODE_PERSISTENT, MODE_TREE = 0, 1, 2, 3

R_NOT_READY, R_OUT_OF_DISK, R_NET_UNAVAIL, R_UNSCHEDULABLE = 0, 1, 2, 3
R_PODS, R_CPU, R_MEMORY, R_GPU, R_EPHEMERAL = 4, 5, 6, 7, 8
R_HOSTNAME, R_HOST_PORTS, R_NODE_SELECTOR, R_TAINTS = 9, 10, 11, 12
R_MEM_PRESSURE, R_DISK_PRESSURE, R_LABEL_PRESENCE = 13, 14, 15
R_SCALAR0 = 16
R_POD_AFFINITY, R_EXISTING_ANTI, R_AFFINITY_RULES, R_ANTI_AFFINITY_RULES = 24, 25, 26, 27
R_DISK_CONFLICT, R_MAX_VOLUME_COUNT, R_VOLUME_ZONE, R_SERVICE_AFFINITY = 28, 29, 30, 31

# inter-pod affinity tables (ksim_affinity_tables)
AFF_REQ_AFFINITY, AFF_REQ_ANTI, AFF_PREFERRED = 0, 1, 2
AFF_CARRY_ANTI, AFF_CARRY_PRIO = 0, 1

# volume tables (ksim_volume_tables)
VOL_EBS, VOL_GCE_PD, VOL_AZURE_DISK = 1, 2, 4
VOL_CONFLICT_ANY, VOL_CONFLICT_RW, VOL_READ_ONLY, VOL_NEW, VOL_VIA_PVC = 1, 2, 4, 8, 16

_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_u8p = C.POINTER(C.c_uint8)


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("mode", C.c_int32), ("predicates", C.c_uint32),
                ("weights", C.c_int64 * NW), ("no_priorities", C.c_int32), ("collect_reasons", C.c_int32),
                ("const_score", C.c_int64), ("last_node_index", C.c_uint64)]


class NodeTable(C.Structure):
    _fields_ = [("n_nodes", C.c_int64), ("n_scalar", C.c_int32), ("port_slots", C.c_int32),
                ("alloc_cpu", _i64p), ("alloc_mem", _i64p), ("alloc_gpu", _i64p), ("alloc_eph", _i64p),
                ("allowed_pods", _i32p), ("flags", _u32p), ("label_set", _i32p), ("taint_set", _i32p),
                ("alloc_scalar", _i64p), ("req_cpu", _i64p), ("req_mem", _i64p), ("req_gpu", _i64p),
                ("req_eph", _i64p), ("nz_cpu", _i64p), ("nz_mem", _i64p), ("pod_count", _i32p),
                ("req_scalar", _i64p), ("ports", _u64p), ("port_count", _i32p)]


class ClassTables(C.Structure):
    _fields_ = [("n_classes", C.c_int32), ("n_label_sets", C.c_int32), ("n_taint_sets", C.c_int32),
                ("sel_ok", _u32p), ("taint_ok", _u32p), ("noexec_ok", _u32p), ("tt_class", _u8p),
                ("na_class", _u8p), ("n_tt", _i32p), ("n_na", _i32p), ("tt_val", _i64p), ("na_val", _i64p),
                ("na_add", _i64p), ("svc_ok", _u32p), ("val_width", C.c_int32), ("reserved0", C.c_int32)]


class Pod(C.Structure):
    _fields_ = [("req_cpu", C.c_int64), ("req_mem", C.c_int64), ("req_gpu", C.c_int64), ("req_eph", C.c_int64),
                ("add_cpu", C.c_int64), ("add_mem", C.c_int64), ("add_gpu", C.c_int64), ("add_eph", C.c_int64),
                ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("cls", C.c_int32), ("host", C.c_int32),
                ("flags", C.c_uint32), ("port_off", C.c_int32), ("port_cnt", C.c_int32),
                ("scalar_off", C.c_int32), ("scalar_cnt", C.c_int32), ("aff_ident", C.c_int32),
                ("aff_class", C.c_int32), ("vol_class", C.c_int32), ("reserved", C.c_int32 * 2)]


class ScalarReq(C.Structure):
    _fields_ = [("col", C.c_int32), ("pad", C.c_int32), ("req", C.c_int64), ("add", C.c_int64)]


class Stats(C.Structure):
    _fields_ = [("pods", C.c_int64), ("scheduled", C.c_int64), ("node_evals", C.c_int64),
                ("device_ms", C.c_double), ("kernel_ms", C.c_double), ("kernel_launches", C.c_int64),
                ("mode", C.c_int32), ("blocks", C.c_int32)]


class Result(C.Structure):
    _fields_ = [("node", C.c_int32), ("fit_nodes", C.c_int32), ("last_node_index", C.c_uint64),
                ("reasons", C.c_int32 * NREASONS)]


class NodeRow(C.Structure):
    _fields_ = [("alloc_cpu", C.c_int64), ("alloc_mem", C.c_int64), ("alloc_gpu", C.c_int64), ("alloc_eph", C.c_int64),
                ("allowed_pods", C.c_int32), ("flags", C.c_uint32), ("label_set", C.c_int32), ("taint_set", C.c_int32),
                ("req_cpu", C.c_int64), ("req_mem", C.c_int64), ("req_gpu", C.c_int64), ("req_eph", C.c_int64),
                ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("pod_count", C.c_int32), ("port_count", C.c_int32),
                ("alloc_scalar", _i64p), ("req_scalar", _i64p), ("ports", _u64p)]


SCHEDULE_ONLY, SCHEDULE_ASSUME = 0, 1


class AffinityTables(C.Structure):
    _fields_ = [("n_keys", C.c_int32), ("n_sel", C.c_int32), ("n_ident", C.c_int32), ("n_pair", C.c_int32),
                ("n_carry", C.c_int32), ("n_aclass", C.c_int32), ("n_terms", C.c_int32), ("n_carries", C.c_int32),
                ("n_nodes", C.c_int64), ("cnt_len", C.c_int64), ("carried_len", C.c_int64),
                ("hard_weight", C.c_int32), ("sel_words", C.c_int32), ("carry_words", C.c_int32), ("zone_key", C.c_int32),
                ("dom", _i32p), ("n_dom", _i32p), ("ident_sel", _u64p), ("ident_anti", _u64p), ("ident_prio", _u64p),
                ("pair_sel", _i32p), ("pair_key", _i32p), ("pair_off", _i64p), ("carry_key", _i32p),
                ("carry_kind", _i32p), ("carry_off", _i64p), ("ac", _i32p), ("terms", C.c_void_p),
                ("carries", C.c_void_p), ("cnt", _i32p), ("carried", _i64p), ("spread_pair", _i32p),
                ("aux_pair", _i32p), ("aux_key", C.c_int32), ("aux_kind", C.c_int32), ("aux_weight", C.c_int64),
                ("n_svc", C.c_int32), ("n_svc_labels", C.c_int32), ("svc_ident", C.c_void_p), ("svc_class", _i32p),
                ("svc_miss", C.POINTER(C.c_uint32)), ("svc_conflict", C.POINTER(C.c_uint32)), ("svc_of_off", _i32p),
                ("svc_of", _i32p)]


SVC_LABELS = 8
SVC_IDENT_DTYPE = np.dtype([("pair_all", np.int32), ("pad", np.int32), ("pair_present", np.int32, SVC_LABELS),
                            ("pair_value", np.int32, SVC_LABELS)])


AUX_SPREAD, AUX_SERVICE_ANTI = 0, 1
SHARD_MAX_ZONES = 24   # zones of the spread reduce a node-sharded pass A exchanges (KSIM_PX_ZONES)
SHARD_MAX_AUX_DOMAINS = 24  # the auxiliary priority's domains it exchanges (KSIM_PX_ADOMS)


class VolumeTables(C.Structure):
    _fields_ = [("n_keys", C.c_int32), ("n_vclass", C.c_int32), ("n_refs", C.c_int32), ("vol_slots", C.c_int32),
                ("n_nodes", C.c_int64), ("max_vols", C.c_int32 * 3), ("zone_words", C.c_int32),
                ("key_filter", _u32p), ("vc", _i32p), ("vc_filter", _u32p), ("refs", C.c_void_p),
                ("zone_ok", _u32p), ("slots", _u64p), ("slot_count", _i32p)]


VOL_REF_DTYPE = np.dtype([("key", "<i4"), ("flags", "<u4")])


class NodeState(C.Structure):
    _fields_ = [("req_cpu", _i64p), ("req_mem", _i64p), ("req_gpu", _i64p), ("req_eph", _i64p),
                ("nz_cpu", _i64p), ("nz_mem", _i64p), ("pod_count", _i32p), ("req_scalar", _i64p),
                ("ports", _u64p), ("port_count", _i32p)]


# numpy dtype matching ksim_pod (128 B) so pod queues are built vectorised
POD_DTYPE = np.dtype([("req_cpu", "<i8"), ("req_mem", "<i8"), ("req_gpu", "<i8"), ("req_eph", "<i8"),
                      ("add_cpu", "<i8"), ("add_mem", "<i8"), ("add_gpu", "<i8"), ("add_eph", "<i8"),
                      ("nz_cpu", "<i8"), ("nz_mem", "<i8"), ("cls", "<i4"), ("host", "<i4"), ("flags", "<u4"),
                      ("port_off", "<i4"), ("port_cnt", "<i4"), ("scalar_off", "<i4"), ("scalar_cnt", "<i4"),
                      ("aff_ident", "<i4"), ("aff_class", "<i4"), ("vol_class", "<i4"),
                      ("reserved", "<i4", (2,))])
SCALAR_DTYPE = np.dtype([("col", "<i4"), ("pad", "<i4"), ("req", "<i8"), ("add", "<i8")])
assert POD_DTYPE.itemsize == C.sizeof(Pod) == 128
assert SCALAR_DTYPE.itemsize == C.sizeof(ScalarReq)

EXPORTS = ["ksim_abi_version", "ksim_last_error", "ksim_create", "ksim_destroy", "ksim_load_nodes",
           "ksim_load_classes", "ksim_load_pods", "ksim_schedule", "ksim_evaluate", "ksim_assume",
           "ksim_read_nodes", "ksim_get_counter", "ksim_set_counter", "ksim_selftest", "ksim_sweep",
           "ksim_shard_setup", "ksim_shard_export", "ksim_shard_connect", "ksim_shard_connect_local",
           "ksim_schedule_one", "ksim_pod_add", "ksim_pod_remove", "ksim_node_add", "ksim_node_update",
           "ksim_node_remove", "ksim_node_count", "ksim_append_pods", "ksim_load_affinity", "ksim_load_volumes",
           "ksim_read_volumes", "ksim_grow_volumes"]
IPC_HANDLE_BYTES = 64
MAX_RANKS = 8


class KsimError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("ksim error %d: %s" % (code, msg))
        self.code = code


class KsimUnsupported(KsimError):
    pass


class NoNodesAvailable(KsimError):
    """core.ErrNoNodesAvailable (generic_scheduler.go:64): "no nodes available to schedule pods"."""


_lib = None


def lib():
    """Load libksim.so (raises if it was not built — the product has no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libksim.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    L.ksim_abi_version.restype = C.c_int
    L.ksim_last_error.restype = C.c_char_p
    L.ksim_last_error.argtypes = [C.c_void_p]
    L.ksim_create.argtypes = [C.POINTER(Config), C.POINTER(C.c_void_p)]
    L.ksim_destroy.argtypes = [C.c_void_p]
    L.ksim_destroy.restype = None
    L.ksim_load_nodes.argtypes = [C.c_void_p, C.POINTER(NodeTable)]
    L.ksim_load_classes.argtypes = [C.c_void_p, C.POINTER(ClassTables)]
    L.ksim_load_pods.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]
    L.ksim_schedule.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.POINTER(Stats)]
    L.ksim_evaluate.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.ksim_assume.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
    L.ksim_read_nodes.argtypes = [C.c_void_p, C.POINTER(NodeState)]
    L.ksim_get_counter.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.ksim_set_counter.argtypes = [C.c_void_p, C.c_uint64]
    L.ksim_selftest.restype = C.c_int
    L.ksim_shard_setup.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int64]
    L.ksim_shard_export.argtypes = [C.c_void_p, C.c_void_p]
    L.ksim_shard_connect.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    L.ksim_shard_connect_local.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    L.ksim_sweep.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                             C.POINTER(Stats)]
    podargs = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]
    L.ksim_schedule_one.argtypes = [C.c_void_p] + podargs + [C.c_int32, C.POINTER(Result)]
    L.ksim_pod_add.argtypes = [C.c_void_p, C.c_int64] + podargs
    L.ksim_pod_remove.argtypes = [C.c_void_p, C.c_int64] + podargs
    L.ksim_node_add.argtypes = [C.c_void_p, C.c_int64, C.POINTER(NodeRow)]
    L.ksim_node_update.argtypes = [C.c_void_p, C.c_int64, C.POINTER(NodeRow)]
    L.ksim_node_remove.argtypes = [C.c_void_p, C.c_int64]
    L.ksim_node_count.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    L.ksim_append_pods.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]
    L.ksim_load_affinity.argtypes = [C.c_void_p, C.POINTER(AffinityTables)]
    L.ksim_load_volumes.argtypes = [C.c_void_p, C.POINTER(VolumeTables)]
    L.ksim_grow_volumes.argtypes = [C.c_void_p, C.POINTER(VolumeTables)]
    L.ksim_read_volumes.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    if L.ksim_abi_version() != ABI_VERSION:
        raise ImportError("libksim.so ABI version mismatch")
    _lib = L
    return L


def ptr(a, ctype):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))


def vptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class Handle:
    """RAII wrapper around ksim_handle* (one per device / host thread)."""

    def __init__(self, cfg: Config):
        self._L = lib()
        h = C.c_void_p()
        self._check(self._L.ksim_create(C.byref(cfg), C.byref(h)), None)
        self.h = h
        self._keep = []

    @classmethod
    def adopt(cls, h, cfg=None):
        """Wrap a handle another entry point created (ksim_k8s_open); it is destroyed with this."""
        self = cls.__new__(cls)
        self._L = lib()
        self.h = h
        self._keep = []
        return self

    def _check(self, rc, h):
        if rc != KSIM_OK:
            msg = self._L.ksim_last_error(h).decode(errors="replace")
            cls = KsimUnsupported if rc == E_UNSUPPORTED else (NoNodesAvailable if rc == E_NO_NODES else KsimError)
            raise cls(rc, msg)

    def call(self, fn, *args):
        self._check(getattr(self._L, fn)(self.h, *args), self.h)

    def close(self):
        if getattr(self, "h", None):
            self._L.ksim_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
