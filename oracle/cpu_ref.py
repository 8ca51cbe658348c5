"""ORACLE — test infrastructure only.  ctypes wrapper of oracle/build/libksim_ref.so
(cpu_ref.c, the table-level C restatement).  Used by tests/ as the large-scale checker
and by bench.py as the cpu_baseline leg; never by the product path."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libksim_ref.so")
_lib = None


class Extra(C.Structure):
    """ksim_ref_extra (cpu_ref.c): the mutable affinity counts and volume slots."""
    _fields_ = [("cnt", C.POINTER(C.c_int32)), ("carried", C.POINTER(C.c_int64)),
                ("vslots", C.POINTER(C.c_uint64)), ("vcount", C.POINTER(C.c_int32)),
                ("svc_conflict", C.POINTER(C.c_uint32)), ("svc_err", C.c_int32), ("pad", C.c_int32)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError("oracle not built: make -C oracle")
        _lib = C.CDLL(LIB)
        _lib.ksim_ref_run.restype = C.c_int
        _lib.ksim_ref_run_ex.restype = C.c_int
    return _lib


def _state(cluster):
    c = cluster.cols
    return {k: np.ascontiguousarray(c[k]).copy() for k in
            ("req_cpu", "req_mem", "req_gpu", "req_eph", "nz_cpu", "nz_mem", "pod_count", "req_scalar", "ports",
             "port_count")}


def run(cluster, cfg, first=0, count=None, threads=1, state=None, counter=0, tables=None, na_add=None, plan=None,
        extra=None):
    """Schedule cluster pods [first, first+count) on the CPU.  `state` (dict of dynamic
    columns, updated in place) defaults to a fresh copy of the cluster's initial state.
    tables / na_add: a scheduler's class tables and NodePreferAvoidPods addends
    (scheduler.class_tables_for), default the cluster's own tables.  plan: a scheduler.Plan —
    its config, class tables, node flags, pod queue and affinity / volume tables are used instead
    (the table-level view of exactly what the device loads); `extra` (dict: cnt, carried, vslots,
    vcount, updated in place) then carries the affinity counts / volume slots between calls.
    Returns (out_node, reasons, state, counter) — plus the extra dict when a plan is given."""
    from ksim import abi  # ABI struct layouts (include/ksim.h)
    from ksim.ingest import class_tables_struct

    if plan is not None:
        cfg, tables, na_add, pods = plan.cfg, plan.tables, plan.na_add, np.ascontiguousarray(plan.pods)
    else:
        pods = np.ascontiguousarray(cluster.pods)
    count = len(pods) - first if count is None else count
    if state is None:
        state = _state(cluster)
    st = abi.NodeState()
    for k, ct in (("req_cpu", C.c_int64), ("req_mem", C.c_int64), ("req_gpu", C.c_int64), ("req_eph", C.c_int64),
                  ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("pod_count", C.c_int32), ("req_scalar", C.c_int64),
                  ("ports", C.c_uint64), ("port_count", C.c_int32)):
        setattr(st, k, abi.ptr(state[k], ct))
    tab = cluster.node_table()
    if plan is not None and plan.flags is not None:
        tab.flags = abi.ptr(plan.flags, C.c_uint32)
    ct = class_tables_struct(cluster.tables if tables is None else tables, na_add)
    out = np.zeros(count, np.int32)
    reasons = np.zeros((count, abi.NREASONS), np.int32)
    ctr = C.c_uint64(counter)
    if plan is None:
        rc = lib().ksim_ref_run(C.byref(cfg), C.byref(tab), C.byref(st), C.byref(ct), abi.vptr(pods),
                                abi.vptr(cluster.pod_ports), abi.vptr(cluster.pod_scalars), C.c_int64(first),
                                C.c_int64(count), C.c_int(threads), abi.vptr(out), abi.vptr(reasons), C.byref(ctr))
        if rc != 0:
            raise RuntimeError("ksim_ref_run failed: %d" % rc)
        return out, reasons, state, ctr.value
    at = vt = None
    if extra is None:
        extra = {}
        if plan.affinity is not None:
            extra["cnt"] = np.ascontiguousarray(plan.affinity["cnt"]).copy()
            extra["carried"] = np.ascontiguousarray(plan.affinity["carried"]).copy()
            if plan.affinity.get("svc_on") and plan.affinity.get("svc_use", True):
                extra["svc_conflict"] = np.ascontiguousarray(plan.affinity["svc_conflict"], np.uint32).copy()
        if plan.volumes is not None:
            extra["vslots"] = np.ascontiguousarray(plan.volumes["slots"]).copy()
            extra["vcount"] = np.ascontiguousarray(plan.volumes["slot_count"]).copy()
    x = Extra()
    if plan.affinity is not None:
        from ksim.affinity import tables_struct
        at = tables_struct(plan.affinity)
        x.cnt = abi.ptr(extra["cnt"], C.c_int32)
        x.carried = abi.ptr(extra["carried"], C.c_int64)
        if "svc_conflict" in extra:
            x.svc_conflict = abi.ptr(extra["svc_conflict"], C.c_uint32)
    if plan.volumes is not None:
        from ksim.volumes import tables_struct as vol_struct
        vt = vol_struct(plan.volumes, plan.use_zone)
        x.vslots = abi.ptr(extra["vslots"], C.c_uint64)
        x.vcount = abi.ptr(extra["vcount"], C.c_int32)
    rc = lib().ksim_ref_run_ex(C.byref(cfg), C.byref(tab), C.byref(st), C.byref(ct),
                               C.byref(at) if at is not None else None, C.byref(vt) if vt is not None else None,
                               C.byref(x), abi.vptr(pods), abi.vptr(cluster.pod_ports), abi.vptr(cluster.pod_scalars),
                               C.c_int64(first), C.c_int64(count), C.c_int(threads), abi.vptr(out), abi.vptr(reasons),
                               C.byref(ctr))
    if rc == -4:
        raise Unsupported("ksim_ref_run_ex: KSIM_E_UNSUPPORTED (CheckServiceAffinity lenders disagree)")
    if rc != 0:
        raise RuntimeError("ksim_ref_run_ex failed: %d" % rc)
    return out, reasons, state, ctr.value, extra


class Unsupported(RuntimeError):
    """The oracle refuses the run where the library does (KSIM_E_UNSUPPORTED)."""
