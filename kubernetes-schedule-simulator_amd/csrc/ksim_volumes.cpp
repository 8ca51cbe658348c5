// ksim_volumes.cpp — ksim_load_volumes / ksim_read_volumes: validates and uploads the volume
// tables (layout in include/ksim.h; built by ksim/volumes.py) that NoDiskConflict
// (predicates.go:220-285), the MaxPD volume counts (:313-507) and NoVolumeZoneConflict (:539-633)
// read on the device (ksim_common.h ksim_disk_conflict / ksim_max_volumes / ksim_vol_zone_ok), and
// that every commit / release of a volume pod updates (ksim_vol_commit).
//
// Every index the kernels follow is checked here against the array it indexes, so a malformed
// table is a KSIM_E_INVAL on the host, never an out-of-bounds access on the device.
#include "ksim_handle.h"

namespace {

// (k0, j0, c0): the keys, refs and volume classes already checked (an in-place grow: the header's
// contract keeps existing entries unchanged, so only the new ones are checked)
int validate(ksim_handle* h, const ksim_volume_tables* t, bool keep, int32_t k0 = 0, int32_t j0 = 0, int32_t c0 = 0) {
  const int64_t n = h->ctx.n;
  if (t->n_nodes != n)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: tables for %lld nodes, table has %lld", (long long)t->n_nodes,
                     (long long)n);
  if (t->n_keys < 0 || t->n_vclass < 0 || t->n_refs < 0 || t->vol_slots < 0 || t->zone_words < 0)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: negative size");
  if (t->vol_slots > 65535)
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_load_volumes: more than 65535 volume slots per node");
  for (int k = 0; k < 3; ++k)
    if (t->max_vols[k] < 0) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: negative volume limit");
  auto need = [&](const void* p, int64_t cnt) { return cnt == 0 || p != nullptr; };
  if (!need(t->key_filter, t->n_keys) || !need(t->vc, 2 * (int64_t)t->n_vclass) || !need(t->vc_filter, t->n_vclass) ||
      !need(t->refs, t->n_refs) || (!keep && (!need(t->slots, (int64_t)t->vol_slots * n) || !need(t->slot_count, n))))
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: missing array");
  if (keep && (t->n_keys < h->vol_n_keys || t->n_vclass < h->vol_n_class || t->vol_slots < h->vol_h.vol_slots))
    return ksim_fail(h, KSIM_E_INVAL, "ksim_grow_volumes: the tables may only grow (keys %d < %d, classes %d < %d or "
                     "slots %d < %d)", t->n_keys, h->vol_n_keys, t->n_vclass, h->vol_n_class, t->vol_slots,
                     h->vol_h.vol_slots);
  if (t->zone_ok && t->zone_words != (h->n_label_sets + 31) / 32)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: zone_words does not match the %d loaded label sets",
                     h->n_label_sets);
  for (int32_t k = k0; k < t->n_keys; ++k)
    if (t->key_filter[k] & ~(KSIM_VOL_EBS | KSIM_VOL_GCE_PD | KSIM_VOL_AZURE_DISK))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: key %d has unknown filter bits", k);
  const uint32_t ref_bits = KSIM_VOL_CONFLICT_ANY | KSIM_VOL_CONFLICT_RW | KSIM_VOL_READ_ONLY | KSIM_VOL_NEW | KSIM_VOL_VIA_PVC;
  for (int32_t j = j0; j < t->n_refs; ++j)
    if (t->refs[j].key < 0 || t->refs[j].key >= t->n_keys || (t->refs[j].flags & ~ref_bits))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: ref %d out of range", j);
  for (int32_t c = c0; c < t->n_vclass; ++c) {
    const int64_t off = t->vc[2 * (int64_t)c], cnt = t->vc[2 * (int64_t)c + 1];
    if (off < 0 || cnt < 0 || off + cnt > t->n_refs)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: class %d refs out of bounds", c);
  }
  for (int64_t i = 0; !keep && i < n; ++i) {
    const int32_t cnt = t->slot_count[i];
    if (cnt < 0 || cnt > t->vol_slots)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: node %lld slot count out of range", (long long)i);
    for (int32_t s = 0; s < cnt; ++s) {
      const uint64_t w = t->slots[(int64_t)s * n + i];
      const int64_t key = (int64_t)(w >> 32);
      if (key >= t->n_keys || (w & 0xFFFFFFFFull) == 0)
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: node %lld slot %d holds no mount of a known key",
                         (long long)i, s);
    }
  }
  for (size_t q = 0; c0 == 0 && q < h->q_vclass.size(); ++q)
    if (h->q_vclass[q] > t->n_vclass)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: queued pod %zu uses a volume class beyond the tables", q);
  return KSIM_OK;
}

}  // namespace

// keep: ksim_grow_volumes — the device's mounts stay (re-laid out when vol_slots grew).
static int load(ksim_handle* h, const ksim_volume_tables* t, bool keep) {
  if (!h || !t) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: null argument");
  if (!h->have_nodes || !h->have_classes) return ksim_fail(h, KSIM_E_STATE, "ksim_load_volumes: load nodes and classes first");
  if (keep && (!h->have_vol || h->vol_stale))
    return ksim_fail(h, KSIM_E_STATE, "ksim_grow_volumes: no current volume tables (load them after a node event)");
  HIPCHK(h, hipSetDevice(h->device));
  const int64_t n = h->ctx.n;
  VolSeg& sg = h->vol_seg;
  // A grow within the segments' capacities, with the same mounts and zone words: only the entries
  // past the loaded counts are checked, written into the host mirror and uploaded (the descriptor,
  // which holds no counts, and every earlier entry stay) — O(new entries), not O(cached pods).
  if (keep && sg.valid && t->vol_slots == h->vol_h.vol_slots && t->n_keys <= sg.cap_keys && t->n_vclass <= sg.cap_vclass &&
      t->n_refs <= sg.cap_refs && t->zone_words == h->vol_h.zone_words && (t->zone_ok != nullptr) == (h->vol_h.zone_ok != nullptr) &&
      t->max_vols[0] == h->vol_h.max_vols[0] && t->max_vols[1] == h->vol_h.max_vols[1] && t->max_vols[2] == h->vol_h.max_vols[2]) {
    const int32_t k0 = h->vol_n_keys, c0 = h->vol_n_class, j0 = sg.n_refs;
    if (t->n_refs < j0) return ksim_fail(h, KSIM_E_INVAL, "ksim_grow_volumes: the tables may only grow (refs %d < %d)", t->n_refs, j0);
    int rc = validate(h, t, keep, k0, j0, c0);
    if (rc) return rc;
    std::vector<char>& hb = h->vol_small_host;
    struct Part { size_t off, esz; const void* src; int64_t from, to; };
    const int32_t zw = t->zone_ok ? t->zone_words : 0;
    const Part parts[] = {{sg.o_kf, 4, t->key_filter, k0, t->n_keys},
                          {sg.o_vc, 8, t->vc, c0, t->n_vclass},  // (two int32 per class)
                          {sg.o_vf, 4, t->vc_filter, c0, t->n_vclass},
                          {sg.o_refs, sizeof(ksim_vol_ref), t->refs, j0, t->n_refs},
                          {sg.o_zo, (size_t)zw * 4, t->zone_ok, c0, zw ? t->n_vclass : c0}};
    const bool side = h->serve_live.load();
    if (side && !h->side_stream) HIPCHK(h, hipStreamCreateWithFlags(&h->side_stream, hipStreamNonBlocking));
    hipStream_t st = side ? h->side_stream : ksim_stream(h);
    for (const Part& x : parts) {
      if (x.to <= x.from || !x.esz) continue;
      const size_t a = x.off + (size_t)x.from * x.esz, b = (size_t)(x.to - x.from) * x.esz;
      memcpy(hb.data() + a, static_cast<const char*>(x.src) + (size_t)x.from * x.esz, b);
      HIPCHK(h, hipMemcpyAsync(h->vol_small + a, hb.data() + a, b, hipMemcpyHostToDevice, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    if (side) h->serve_shared = true;  // (the resident kernel's next message acquires the new entries)
    h->vol_in_place += side ? 1 : 0;
    h->vol_n_class = t->n_vclass;
    h->vol_n_keys = t->n_keys;
    sg.n_refs = t->n_refs;
    for (int32_t c = c0; c < t->n_vclass; ++c) h->vol_max_ref = std::max(h->vol_max_ref, t->vc[2 * (int64_t)c + 1]);
    return KSIM_OK;
  }
  int rc = validate(h, t, keep);
  if (rc) return rc;
  // the small tables, packed: [KsimVol][key_filter][vc][vc_filter][refs][zone_ok], 16-byte aligned
  size_t off = 0;
  auto seg = [&](size_t bytes) {
    const size_t o = off;
    off = (off + bytes + 15) & ~(size_t)15;
    return o;
  };
  // segment capacities: exact for a load, doubled for a grow (the next grows then go in place)
  const int64_t f = keep ? 2 : 1;
  const int64_t ck = std::max<int64_t>((int64_t)t->n_keys * f, 1), cv = std::max<int64_t>((int64_t)t->n_vclass * f, 1),
                cr = std::max<int64_t>((int64_t)t->n_refs * f, 1);
  const size_t o_V = seg(sizeof(KsimVol)), o_kf = seg(sizeof(*t->key_filter) * ck),
               o_vc = seg(sizeof(*t->vc) * 2 * (size_t)cv), o_vf = seg(sizeof(*t->vc_filter) * cv),
               o_refs = seg(sizeof(*t->refs) * cr),
               o_zo = seg(t->zone_ok ? sizeof(*t->zone_ok) * (size_t)cv * t->zone_words : 0);
  char* old_small = nullptr;
  if (off > h->vol_small_cap) {  // grown geometrically: most grows reuse the buffer
    old_small = h->vol_small;
    const size_t cap = std::max<size_t>(off * 2, 4096);
    char* q;
    if ((rc = dev_alloc(h, &q, cap))) return rc;
    h->vol_small = q;
    h->vol_small_cap = cap;
  }
  char* base = h->vol_small;
  std::vector<char>& hb = h->vol_small_host;  // kept until the next load: the upload reads it
  hb.assign(off, 0);
  auto put = [&](size_t o, const void* src, size_t bytes) {
    if (bytes) memcpy(hb.data() + o, src, bytes);
  };
  put(o_kf, t->key_filter, sizeof(*t->key_filter) * t->n_keys);
  put(o_vc, t->vc, sizeof(*t->vc) * 2 * (size_t)t->n_vclass);
  put(o_vf, t->vc_filter, sizeof(*t->vc_filter) * t->n_vclass);
  put(o_refs, t->refs, sizeof(*t->refs) * t->n_refs);
  if (t->zone_ok) put(o_zo, t->zone_ok, sizeof(*t->zone_ok) * (size_t)t->n_vclass * t->zone_words);
  KsimVol V{};
  uint64_t* slots;
  int32_t* sc;
  const size_t nb0 = h->bufs.size();
  const bool carry = keep && t->vol_slots == h->vol_h.vol_slots;  // the mounts stay where they are
  if (!keep) {
    if ((rc = dev_upload(h, &slots, t->slots, (size_t)t->vol_slots * n)) || (rc = dev_upload(h, &sc, t->slot_count, n)))
      return rc;
  } else if (carry) {
    slots = h->vol_h.slots;
    sc = h->vol_h.slot_count;
  } else {  // [S][n] → [S'][n]: the first S rows are one contiguous block
    if ((rc = dev_alloc(h, &slots, (size_t)t->vol_slots * n)) || (rc = dev_alloc(h, &sc, (size_t)n))) return rc;
    HIPCHK(h, hipMemsetAsync(slots, 0, (size_t)t->vol_slots * n * 8, ksim_stream(h)));
    HIPCHK(h, hipMemcpyAsync(slots, h->vol_h.slots, (size_t)h->vol_h.vol_slots * n * 8, hipMemcpyDeviceToDevice, ksim_stream(h)));
    HIPCHK(h, hipMemcpyAsync(sc, h->vol_h.slot_count, (size_t)n * 4, hipMemcpyDeviceToDevice, ksim_stream(h)));
  }
  V.n = n;
  V.slots = slots; V.slot_count = sc;
  V.key_filter = reinterpret_cast<const uint32_t*>(base + o_kf);
  V.vc = reinterpret_cast<const int32_t*>(base + o_vc);
  V.vc_filter = reinterpret_cast<const uint32_t*>(base + o_vf);
  V.refs = reinterpret_cast<const ksim_vol_ref*>(base + o_refs);
  V.zone_ok = t->zone_ok ? reinterpret_cast<const uint32_t*>(base + o_zo) : nullptr;
  for (int k = 0; k < 3; ++k) V.max_vols[k] = t->max_vols[k];
  V.vol_slots = t->vol_slots;
  V.zone_words = t->zone_words;
  put(o_V, &V, sizeof V);
  // a grow in place (same buffers, same mounts) beside a running resident per-pod kernel: on the
  // side stream (the kernel reads no volume table between messages) and the next message acquires
  const bool side = carry && !old_small && h->serve_live.load();
  if (side && !h->side_stream) HIPCHK(h, hipStreamCreateWithFlags(&h->side_stream, hipStreamNonBlocking));
  HIPCHK(h, hipMemcpyAsync(base, hb.data(), off, hipMemcpyHostToDevice, side ? h->side_stream : ksim_stream(h)));
  if (side) {
    HIPCHK(h, hipStreamSynchronize(h->side_stream));
    h->serve_shared = true;
    h->vol_in_place += 1;
  }
  KsimVol* dev = reinterpret_cast<KsimVol*>(base);
  std::vector<void*> fresh;  // this load's mount buffers (taken before any free shifts h->bufs)
  for (size_t k = nb0; k < h->bufs.size(); ++k) fresh.push_back(h->bufs[k].p);
  if (carry) { fresh.push_back(slots); fresh.push_back(sc); }
  const bool frees = old_small || !carry;
  if (frees) HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  for (void* q : h->vol_bufs)  // the previous mounts (reload / re-layout), unless carried over
    if (!(carry && (q == (void*)slots || q == (void*)sc))) dev_free(h, q);
  if (old_small) dev_free(h, old_small);
  h->vol_bufs = fresh;
  const bool moved = dev != h->vol_dev;
  h->vol_dev = dev;
  h->vol_h = V;
  h->ctx.vol = dev;
  h->vol_n_class = t->n_vclass;
  h->vol_n_keys = t->n_keys;
  sg = VolSeg{true, ck, cv, cr, t->n_refs, o_kf, o_vc, o_vf, o_refs, o_zo};
  h->vol_max_ref = 0;
  for (int32_t c = 0; c < t->n_vclass; ++c) h->vol_max_ref = std::max(h->vol_max_ref, t->vc[2 * (int64_t)c + 1]);
  h->have_vol = true;
  h->vol_stale = false;
  // the table pointer is baked into the launch graph's kernel arguments
  if (moved && h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
  if (moved && h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
  return KSIM_OK;
}

extern "C" int ksim_load_volumes(ksim_handle* h, const ksim_volume_tables* t) { return load(h, t, false); }

// Grow the tables the pod-side lookups index (keys, volume classes, refs, zone verdicts, more
// slots per node) while the device keeps every node's mounts: the per-pod path's answer to a pod
// that brings new volumes (its cost is the small tables, not O(cached pods)).
extern "C" int ksim_grow_volumes(ksim_handle* h, const ksim_volume_tables* t) { return load(h, t, true); }

extern "C" int ksim_read_volumes(ksim_handle* h, uint64_t* slots, int32_t* slot_count) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "ksim_read_volumes: null handle");
  if (!h->have_vol) return ksim_fail(h, KSIM_E_STATE, "ksim_read_volumes: no volume tables loaded");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  const KsimVol& V = h->vol_h;
  if (slots && V.vol_slots)
    HIPCHK(h, hipMemcpy(slots, V.slots, (size_t)V.vol_slots * V.n * 8, hipMemcpyDeviceToHost));
  if (slot_count && V.n) HIPCHK(h, hipMemcpy(slot_count, V.slot_count, (size_t)V.n * 4, hipMemcpyDeviceToHost));
  return KSIM_OK;
}
