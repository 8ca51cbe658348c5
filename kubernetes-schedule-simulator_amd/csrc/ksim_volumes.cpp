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

int validate(ksim_handle* h, const ksim_volume_tables* t) {
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
      !need(t->refs, t->n_refs) || !need(t->slots, (int64_t)t->vol_slots * n) || !t->slot_count)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: missing array");
  if (t->zone_ok && t->zone_words != (h->n_label_sets + 31) / 32)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: zone_words does not match the %d loaded label sets",
                     h->n_label_sets);
  for (int32_t k = 0; k < t->n_keys; ++k)
    if (t->key_filter[k] & ~(KSIM_VOL_EBS | KSIM_VOL_GCE_PD | KSIM_VOL_AZURE_DISK))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: key %d has unknown filter bits", k);
  const uint32_t ref_bits = KSIM_VOL_CONFLICT_ANY | KSIM_VOL_CONFLICT_RW | KSIM_VOL_READ_ONLY | KSIM_VOL_NEW | KSIM_VOL_VIA_PVC;
  for (int32_t j = 0; j < t->n_refs; ++j)
    if (t->refs[j].key < 0 || t->refs[j].key >= t->n_keys || (t->refs[j].flags & ~ref_bits))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: ref %d out of range", j);
  for (int32_t c = 0; c < t->n_vclass; ++c) {
    const int64_t off = t->vc[2 * (int64_t)c], cnt = t->vc[2 * (int64_t)c + 1];
    if (off < 0 || cnt < 0 || off + cnt > t->n_refs)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: class %d refs out of bounds", c);
  }
  for (int64_t i = 0; i < n; ++i) {
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
  for (size_t q = 0; q < h->q_vclass.size(); ++q)
    if (h->q_vclass[q] > t->n_vclass)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: queued pod %zu uses a volume class beyond the tables", q);
  return KSIM_OK;
}

}  // namespace

extern "C" int ksim_load_volumes(ksim_handle* h, const ksim_volume_tables* t) {
  if (!h || !t) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_volumes: null argument");
  if (!h->have_nodes || !h->have_classes) return ksim_fail(h, KSIM_E_STATE, "ksim_load_volumes: load nodes and classes first");
  if (h->shard.world > 1) return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_load_volumes: not available on a node-sharded handle");
  HIPCHK(h, hipSetDevice(h->device));
  int rc = validate(h, t);
  if (rc) return rc;
  const int64_t n = h->ctx.n;
  const size_t nb0 = h->bufs.size();
  KsimVol V{};
  uint32_t *kf, *vf, *zo = nullptr;
  int32_t *vc, *sc;
  ksim_vol_ref* refs;
  uint64_t* slots;
  if ((rc = dev_upload(h, &kf, t->key_filter, t->n_keys)) || (rc = dev_upload(h, &vc, t->vc, 2 * (size_t)t->n_vclass)) ||
      (rc = dev_upload(h, &vf, t->vc_filter, t->n_vclass)) || (rc = dev_upload(h, &refs, t->refs, t->n_refs)) ||
      (rc = dev_upload(h, &slots, t->slots, (size_t)t->vol_slots * n)) || (rc = dev_upload(h, &sc, t->slot_count, n)))
    return rc;
  if (t->zone_ok && (rc = dev_upload(h, &zo, t->zone_ok, (size_t)t->n_vclass * t->zone_words))) return rc;
  V.n = n;
  V.slots = slots; V.slot_count = sc; V.key_filter = kf; V.vc = vc; V.vc_filter = vf; V.refs = refs; V.zone_ok = zo;
  for (int k = 0; k < 3; ++k) V.max_vols[k] = t->max_vols[k];
  V.vol_slots = t->vol_slots;
  V.zone_words = t->zone_words;
  KsimVol* dev;
  if ((rc = dev_upload(h, &dev, &V, 1))) return rc;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  for (void* q : h->vol_bufs) dev_free(h, q);  // the previous tables (reload)
  h->vol_bufs.clear();
  for (size_t k = nb0; k < h->bufs.size(); ++k) h->vol_bufs.push_back(h->bufs[k].p);
  h->vol_dev = dev;
  h->vol_h = V;
  h->ctx.vol = dev;
  h->vol_n_class = t->n_vclass;
  h->vol_max_ref = 0;
  for (int32_t c = 0; c < t->n_vclass; ++c) h->vol_max_ref = std::max(h->vol_max_ref, t->vc[2 * (int64_t)c + 1]);
  h->have_vol = true;
  h->vol_stale = false;
  // the table pointer is baked into the launch graph's kernel arguments
  if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
  if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
  return KSIM_OK;
}

extern "C" int ksim_read_volumes(ksim_handle* h, uint64_t* slots, int32_t* slot_count) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "ksim_read_volumes: null handle");
  if (!h->have_vol) return ksim_fail(h, KSIM_E_STATE, "ksim_read_volumes: no volume tables loaded");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const KsimVol& V = h->vol_h;
  if (slots && V.vol_slots)
    HIPCHK(h, hipMemcpy(slots, V.slots, (size_t)V.vol_slots * V.n * 8, hipMemcpyDeviceToHost));
  if (slot_count && V.n) HIPCHK(h, hipMemcpy(slot_count, V.slot_count, (size_t)V.n * 4, hipMemcpyDeviceToHost));
  return KSIM_OK;
}
