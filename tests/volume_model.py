"""Plain-Python model of the kernels' volume evaluation over the ksim_volume_tables arrays
(ksim_common.h ksim_disk_conflict / ksim_max_volumes / ksim_vol_zone_ok / ksim_vol_commit), so the
tables ksim/volumes.py builds can be checked against the object oracle without a GPU.  Test
infrastructure only."""
from ksim import abi

RW, RO, PV = (0, 0x7FF), (11, 0x7FF), (22, 0x3FF)


def slots_of(d, i):
    """Node i's mounts: {key: [rw, ro, pvc]}."""
    out = {}
    for s in range(int(d["slot_count"][i])):
        w = int(d["slots"][s, i])
        out[w >> 32] = [w & 0x7FF, (w >> 11) & 0x7FF, (w >> 22) & 0x3FF]
    return out


def refs_of(d, vclass):
    off, cnt = (int(x) for x in d["vc"][vclass - 1])
    return [(int(r["key"]), int(r["flags"])) for r in d["refs"][off:off + cnt]]


def disk_conflict(d, vclass, mounts):
    for k, f in refs_of(d, vclass):
        if not f & (abi.VOL_CONFLICT_ANY | abi.VOL_CONFLICT_RW) or k not in mounts:
            continue
        rw, ro, _ = mounts[k]
        if (rw + ro > 0) if f & abi.VOL_CONFLICT_ANY else rw > 0:
            return True
    return False


def max_volume_fail(d, vclass, mounts, which):
    want = int(d["vc_filter"][vclass - 1]) & which
    kf = d["key_filter"]
    for t in range(3):
        f = 1 << t
        if not want & f:
            continue
        have = sum(1 for k in mounts if int(kf[k]) & f)
        add = sum(1 for k, fl in refs_of(d, vclass) if fl & abi.VOL_NEW and int(kf[k]) & f and k not in mounts)
        if have + add > d["max_vols"][t]:
            return True
    return False


def zone_ok(d, vclass, label_set):
    if not d["zone_words"]:
        return True
    return bool((int(d["zone_ok"][vclass - 1, label_set >> 5]) >> (label_set & 31)) & 1)


def commit(mounts, d, vclass, sign=1):
    for k, f in refs_of(d, vclass):
        j = 2 if f & abi.VOL_VIA_PVC else 1 if f & abi.VOL_READ_ONLY else 0
        m = mounts.setdefault(k, [0, 0, 0])
        m[j] += sign
        if sum(m) == 0:
            del mounts[k]
