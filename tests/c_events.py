"""Event scripts for tests/c/ksim_k8s_events.c: a seeded informer-style stream (tests/events.py)
flattened exactly as a Go adapter would flatten v1 objects (ksim/frontend.py flatten_node /
flatten_pod → the ksim_k8s_* structs) and written as tokens in the structs' field order (integers;
strings percent-encoded, "-" for "", "~" for NULL; arrays as a count then the elements)."""
from ksim import frontend

_SAFE = set(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789._/:")


def _s(x):
    if x is None:
        return "~"
    if x == b"":
        return "-"
    return "".join(chr(b) if b in _SAFE else "%%%02X" % b for b in x)


def _arr(n, ptr, fn):
    return [str(n)] + [t for i in range(n) for t in fn(ptr[i])]


def _kv(x):
    return [_s(x.key), _s(x.value)]


def _req(x):
    return [_s(x.key), _s(x.op)] + _arr(x.n_values, x.values, lambda v: [_s(v)])


def _node_term(x):
    return _arr(x.n_reqs, x.reqs, _req)


def _label_selector(x):
    return [str(x.present)] + _arr(x.n_match_labels, x.match_labels, _kv) + _arr(x.n_exprs, x.exprs, _req)


def _pod_term(x):
    return (_label_selector(x.selector) + _arr(x.n_namespaces, x.namespaces, lambda v: [_s(v)]) +
            [_s(x.topology_key), str(x.weight)])


def _container(x):
    return ([str(x.has_cpu), str(x.has_mem), str(x.cpu_milli), str(x.mem), str(x.gpu), str(x.eph)] +
            _arr(x.n_other, x.other, lambda r: [_s(r.name), str(r.value)]) + [str(x.qos_positive)] +
            _arr(x.n_ports, x.ports, lambda p: [_s(p.host_ip), _s(p.protocol), str(p.host_port)]) + [_s(x.image)])


def _volume(x):
    return [str(x.kind), str(x.read_only), _s(x.id), _s(x.pool), _s(x.image)] + _arr(x.n_monitors, x.monitors, lambda v: [_s(v)])


def pod_tokens(x):
    t = [_s(x.name), _s(x.namespace_)] + _arr(x.n_labels, x.labels, _kv) + [str(x.deleting), _s(x.node_name)]
    t += _arr(x.n_containers, x.containers, _container) + _arr(x.n_init_containers, x.init_containers, _container)
    t += _arr(x.n_node_selector, x.node_selector, _kv) + [str(x.has_node_affinity), str(x.has_required)]
    t += _arr(x.n_required_terms, x.required_terms, _node_term)
    t += _arr(x.n_preferred, x.preferred, lambda p: [str(p.weight)] + _node_term(p.preference))
    t += _arr(x.n_tolerations, x.tolerations, lambda o: [_s(o.key), _s(o.op), _s(o.value), _s(o.effect)])
    t += [str(x.has_pod_affinity), str(x.has_pod_anti_affinity)]
    for n, p in ((x.n_affinity_required, x.affinity_required), (x.n_affinity_preferred, x.affinity_preferred),
                 (x.n_anti_required, x.anti_required), (x.n_anti_preferred, x.anti_preferred)):
        t += _arr(n, p, _pod_term)
    t += _arr(x.n_volumes, x.volumes, _volume)
    t += _arr(x.n_spread, x.spread, _label_selector)
    t += _arr(x.n_spread, x.spread_set_selector, lambda v: [str(v)])
    t += [_s(x.avoid_ctrl_kind), _s(x.avoid_ctrl_uid), _s(x.uid)]
    return t


def node_tokens(x):
    t = [_s(x.name)] + _arr(x.n_labels, x.labels, _kv)
    t += _arr(x.n_taints, x.taints, lambda o: [_s(o.key), _s(o.value), _s(o.effect)]) + [str(x.unschedulable)]
    t += _arr(x.n_conditions, x.conditions, lambda o: [_s(o.type), _s(o.status)])
    t += [str(x.alloc_cpu_milli), str(x.alloc_mem), str(x.alloc_gpu), str(x.alloc_eph), str(x.alloc_pods)]
    t += _arr(x.n_alloc_other, x.alloc_other, lambda r: [_s(r.name), str(r.value)])
    t += _arr(x.n_avoid, x.avoid, lambda a: [str(a.has_controller), _s(a.kind), _s(a.uid)]) + [str(x.has_images)]
    t += _arr(x.n_images, x.images, lambda im: _arr(im.n_names, im.names, lambda v: [_s(v)]) + [str(im.size_bytes)])
    return t


def config_line(cfg, prefer_avoid=0, image_locality=0, hard_weight=10, check_volume_binding=0):
    return " ".join(["CONFIG", str(cfg.device), str(cfg.mode), str(cfg.predicates)] + [str(w) for w in cfg.weights] +
                    [str(cfg.no_priorities), str(cfg.const_score), str(prefer_avoid), str(image_locality), str(hard_weight),
                     str(check_volume_binding)])


def event_line(kind, x, spread=None):
    """One event as a script line; spread: SpreadListers the adapter's listers resolve pods with."""
    k = frontend._Keep()
    pod = lambda p: pod_tokens(frontend.flatten_pod(k, p, frontend.spread_raw(spread, p)))
    node = lambda n: node_tokens(frontend.flatten_node(k, n))
    if kind == "schedule":
        return " ".join(["SCHEDULE"] + pod(x))
    if kind in ("add_node", "remove_node"):
        return " ".join([kind.upper()] + node(x))
    if kind == "update_node":
        return " ".join(["UPDATE_NODE"] + node(x[0]) + node(x[1]))
    if kind == "update_pod":
        return " ".join(["UPDATE_POD"] + pod(x[0]) + pod(x[1]))
    return " ".join([kind.upper()] + pod(x))
