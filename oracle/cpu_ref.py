"""ORACLE — test infrastructure only.  ctypes wrapper of oracle/build/libksim_ref.so
(cpu_ref.c, the table-level C restatement).  Used by tests/ as the large-scale checker
and by bench.py as the cpu_baseline leg; never by the product path."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libksim_ref.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError("oracle not built: make -C oracle")
        _lib = C.CDLL(LIB)
        _lib.ksim_ref_run.restype = C.c_int
    return _lib


def run(cluster, cfg, first=0, count=None, threads=1, state=None, counter=0, tables=None, na_add=None):
    """Schedule cluster pods [first, first+count) on the CPU.  `state` (dict of dynamic
    columns, updated in place) defaults to a fresh copy of the cluster's initial state.
    tables / na_add: a scheduler's class tables and NodePreferAvoidPods addends
    (scheduler.class_tables_for), default the cluster's own tables.
    Returns (out_node, reasons, state, counter)."""
    from ksim import abi  # ABI struct layouts (include/ksim.h)

    n = cluster.n_nodes
    pods = np.ascontiguousarray(cluster.pods)
    count = len(pods) - first if count is None else count
    c = cluster.cols
    if state is None:
        state = {k: np.ascontiguousarray(c[k]).copy() for k in
                 ("req_cpu", "req_mem", "req_gpu", "req_eph", "nz_cpu", "nz_mem", "pod_count", "req_scalar", "ports",
                  "port_count")}
    st = abi.NodeState()
    for k, ct in (("req_cpu", C.c_int64), ("req_mem", C.c_int64), ("req_gpu", C.c_int64), ("req_eph", C.c_int64),
                  ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("pod_count", C.c_int32), ("req_scalar", C.c_int64),
                  ("ports", C.c_uint64), ("port_count", C.c_int32)):
        setattr(st, k, abi.ptr(state[k], ct))
    tab = cluster.node_table()
    from ksim.ingest import class_tables_struct
    ct = class_tables_struct(cluster.tables if tables is None else tables, na_add)
    out = np.zeros(count, np.int32)
    reasons = np.zeros((count, abi.NREASONS), np.int32)
    ctr = C.c_uint64(counter)
    rc = lib().ksim_ref_run(C.byref(cfg), C.byref(tab), C.byref(st), C.byref(ct), abi.vptr(pods),
                            abi.vptr(cluster.pod_ports), abi.vptr(cluster.pod_scalars), C.c_int64(first),
                            C.c_int64(count), C.c_int(threads), abi.vptr(out), abi.vptr(reasons), C.byref(ctr))
    if rc != 0:
        raise RuntimeError("ksim_ref_run failed: %d" % rc)
    return out, reasons, state, ctr.value
