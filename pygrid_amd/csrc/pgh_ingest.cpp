// libpygrid_hip: host bytes -> HBM slab rows: raw diffs, State messages (pageable through the pinned ring, or
// page-locked in one DMA + k_gather_f32), int64 shares as packed varints (k_varint_decode), synthetic
// diffs generated on the device; the FedAvg weights.  Reference: the N x unserialize_model_params loop
// of cycle_manager.py:247-250.
// (struct pgh_ctx and the shared helpers: pgh_ctx.h)
#include "pgh_ctx.h"

using namespace pgh_detail;

// (the public entry points take their C linkage from include/pgh_api.h)

int pgh_ingest_raw(pgh_ctx* c, int client, const void* flat, size_t nbytes, int dtype) {
    if (c && c->grp) return pgh_group_api::ingest_raw(c, client, flat, nbytes, dtype);
    RC(check_dtype(c, dtype));
    if (!flat) return fail(c, PGH_E_ARG, "flat is NULL");
    const size_t es = esize(dtype);
    const size_t whole = (size_t)c->P * es * (size_t)c->parties;  // the whole model: take the slice
    const size_t shard = (size_t)c->pg * es * (size_t)c->parties; // this shard only
    if (nbytes != whole && nbytes != shard)
        return fail(c, PGH_E_ARG, "client %d: got %zu bytes, layout needs %zu (model) or %zu (shard)", client, nbytes,
                    whole, shard);
    DeviceGuard g(c->device);
    int slot = 0;
    RC(claim_slot(c, client, &slot));
    const bool pinned = is_pinned(flat);
    const uint8_t* src = (const uint8_t*)flat;
    const size_t row_elems = nbytes == whole ? (size_t)c->P : (size_t)c->pg;
    const size_t first = nbytes == whole ? (size_t)c->lo : 0;
    for (int s = 0; s < c->parties; ++s)
        RC(stage_h2d(c, row_dest(c, slot, s), src + ((size_t)s * row_elems + first) * es, (size_t)c->pg * es, pinned));
    return mark_ingested(c, client, slot);
}

namespace {
int pinned_gather_ingest(pgh_ctx* c, const uint8_t* pb, const std::vector<Piece>& pieces, int slot, bool ranged);
}

int pgh_ingest_state(pgh_ctx* c, int client, const uint8_t* pb, size_t n) {
    if (c && c->grp) return pgh_group_api::ingest_state(c, client, pb, n);
    RC(check_dtype(c, PGH_F32));
    if (!pb && n) return fail(c, PGH_E_ARG, "pb is NULL");
    // The shard's slice of the payloads goes straight from the protobuf buffer into the pinned ring.
    std::vector<std::pair<size_t, size_t>> spans;
    char what[32];
    snprintf(what, sizeof what, "client %d", client);
    RC(state_shard_spans(c, pb, n, &spans, what));
    std::vector<Piece> pieces;
    for (auto& sp : spans) pieces.push_back(Piece{pb + sp.first, sp.second});
    DeviceGuard g(c->device);
    int slot = 0;
    RC(claim_slot(c, client, &slot));
    // report-time ingest (pgh_set_ingest_ranges): in chunks with an event each, so a close that
    // starts while this DMA is in flight folds each param range as soon as it has landed
    const bool ranged = c->ingest_ranges && !c->streaming && c->pg >= (1 << 20);
    if (n && !pieces.empty() && c->pinned_gather && is_pinned(pb)) {
        // Page-locked message (a report decoded straight into pgh_host_alloc memory,
        // pygrid_amd.report.PinnedPool): no staging copy.  The part of the message holding this
        // shard's payloads goes to HBM in ONE DMA (a few hundred bytes of framing ride along) and
        // k_gather_f32 moves the payloads into the slab row; the call waits for the DMA only (the
        // buffer is borrowed), the gather runs on behind it on the copy stream.
        const double t0 = now_ms();
        RC(pinned_gather_ingest(c, pb, pieces, slot, ranged));
        c->st.h2d_ms_total += now_ms() - t0;
        return mark_ingested(c, client, slot);
    }
    if (n && is_pinned(pb)) {
        // Page-locked message, one DMA per payload piece (PGH_PINNED_GATHER=0).  The buffer is only
        // borrowed for the call, so the call waits for its copies.
        const double t0 = now_ms();
        const Dest d = row_dest(c, slot, 0);
        size_t off = 0;
        for (auto& p : pieces) {
            RC(h2d_range(c, d, (int64_t)(off / 4), p.src, (int64_t)(p.n / 4), c->copy));
            off += p.n;
        }
        CK(c, hipStreamSynchronize(c->copy));
        c->st.h2d_ms_total += now_ms() - t0;
        c->st.h2d_bytes_total += off;
        return mark_ingested(c, client, slot);
    }
    size_t total = 0;
    for (auto& p : pieces) total += p.n;
    if (ranged && total == (size_t)c->pg * 4 && total <= c->pin_slot)
        RC(stage_pieces_h2d_ranged(c, row_dest(c, slot, 0), pieces, total));
    else
        RC(stage_pieces_h2d(c, row_dest(c, slot, 0), pieces));
    return mark_ingested(c, client, slot);
}

namespace {
// One party message of pgh_ingest_state_shares, laid out for HBM: each tensor payload starts
// 16-byte aligned in the device byte buffer and is cut into chunks of VARINT_CHUNK bytes.
struct ShareMsg {
    std::vector<pgh::VChunk> chunks;       // device image of the chunk table (first filled after staging)
    std::vector<const uint8_t*> src;       // host bytes of each chunk
    std::vector<int> span_of;              // tensor of each chunk
    std::vector<pgh_state::VarintStats> st;
    size_t bytes = 0;                      // device buffer bytes (payloads + alignment padding)
    size_t base = 0;                       // where they start in the device buffer
};

int plan_share_msg(pgh_ctx* c, const uint8_t* pb, size_t n, int client, int party, size_t base, ShareMsg* m) {
    std::vector<pgh_state::Span> spans;
    std::string msg;
    int rc = pgh_state::scan_i64(pb, n, &spans, &msg);
    if (rc) return fail(c, rc, "client %d party %d shares State: %s", client, party, msg.c_str());
    if (spans.size() != c->numel.size())
        return fail(c, PGH_E_PARSE, "client %d party %d shares State holds %zu tensors, layout has %zu", client, party,
                    spans.size(), c->numel.size());
    size_t pos = base;  // this party's payloads follow the previous party's in the device buffer
    for (size_t t = 0; t < spans.size(); ++t) {
        const auto& sp = spans[t];
        if (sp.count >= 0 && sp.count != c->numel[t])
            return fail(c, PGH_E_PARSE, "client %d party %d tensor %zu: shape holds %lld values, layout %lld", client,
                        party, t, (long long)sp.count, (long long)c->numel[t]);
        pos = (pos + 15) & ~(size_t)15;
        for (size_t a = 0; a < sp.nbytes; a += pgh::VARINT_CHUNK) {
            const size_t len = std::min(sp.nbytes - a, (size_t)pgh::VARINT_CHUNK);
            m->chunks.push_back(pgh::VChunk{(int64_t)(pos + a), (int64_t)pos, 0, (int32_t)len, 0});
            m->src.push_back(pb + sp.offset + a);
            m->span_of.push_back((int)t);
        }
        pos += sp.nbytes;
    }
    m->bytes = pos - base;
    m->base = base;
    m->st.resize(m->chunks.size());
    return PGH_OK;
}

// After staging: every varint at most 10 bytes and none cut off, per-tensor counts equal to the
// layout; fill each chunk's first flat index.
int check_share_msg(pgh_ctx* c, ShareMsg* m, int client, int party) {
    const size_t T = c->numel.size();
    std::vector<int64_t> count(T, 0);
    int64_t run = 0;  // continuation bytes carried across chunks of one tensor
    int prev_span = -1;
    int64_t flat = 0, span_base = 0;
    for (size_t k = 0; k < m->chunks.size(); ++k) {
        const int t = m->span_of[k];
        const auto& st = m->st[k];
        if (t != prev_span) {
            if (prev_span >= 0 && run)
                return fail(c, PGH_E_PARSE, "client %d party %d tensor %d: int64 payload ends inside a varint", client,
                            party, prev_span);
            for (int u = prev_span + 1; u < t; ++u) span_base += c->numel[(size_t)u];  // empty payloads
            if (prev_span >= 0) span_base += c->numel[(size_t)prev_span];
            run = 0;
            prev_span = t;
            flat = span_base;
        }
        if (st.overlong || run + st.lead > 9)
            return fail(c, PGH_E_PARSE, "client %d party %d tensor %d: varint longer than 10 bytes", client, party, t);
        m->chunks[k].first = flat;
        flat += st.terminators;
        count[(size_t)t] += st.terminators;
        run = st.terminators > 0 ? st.trail : run + st.trail;
    }
    if (run) return fail(c, PGH_E_PARSE, "client %d party %d: int64 payload ends inside a varint", client, party);
    for (size_t t = 0; t < T; ++t)
        if (count[t] != c->numel[t])
            return fail(c, PGH_E_PARSE, "client %d party %d tensor %zu holds %lld int64 values, layout %lld", client,
                        party, t, (long long)count[t], (long long)c->numel[t]);
    return PGH_OK;
}

int grow_device(pgh_ctx* c, void** p, size_t* cap, size_t need, const char* what) {
    if (need <= *cap) return PGH_OK;
    const size_t sz = std::max(need, *cap * 3 / 2);
    CK(c, hipStreamSynchronize(c->copy));  // an earlier decode may still read the old buffer
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, sz) != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, PGH_E_OOM, "%s: device allocation of %zu bytes failed", what, sz);
    }
    *cap = sz;
    return PGH_OK;
}

// Stage one party message: chunk bytes -> pinned ring (copied and counted by the pool threads)
// -> its region of the HBM byte buffer `dev`, on the copy stream.  Nothing is decoded yet.
int stage_share_msg(pgh_ctx* c, ShareMsg& m, uint8_t* dev) {
    const double t0 = now_ms();
    const size_t nk = m.chunks.size();
    size_t k = 0;
    while (k < nk) {
        int ps = 0;
        RC(take_pin_slot(c, &ps));
        const size_t s0 = (size_t)m.chunks[k].off;
        const size_t cap = c->pin_slot;  // whole-slot fills (r01z: smaller fills were slower)
        size_t k1 = k;
        while (k1 < nk && (size_t)m.chunks[k1].off + (size_t)m.chunks[k1].n - s0 <= cap) ++k1;
        if (k1 == k) return fail(c, PGH_E_STATE, "pinned slot smaller than one varint chunk");
        uint8_t* pin = c->h_pin[ps];
        const size_t fill = (size_t)m.chunks[k1 - 1].off + (size_t)m.chunks[k1 - 1].n - s0;
        c->pool_copy->run_items((int)(k1 - k), fill >= (4u << 20), [&](int i) {
            const size_t q = k + (size_t)i;
            uint8_t* dst = pin + ((size_t)m.chunks[q].off - s0);
            m.st[q] = pgh_state::varint_copy_stats(dst, m.src[q], (size_t)m.chunks[q].n);
        });
        ++c->copy_seq;
        CK(c, hipMemcpyAsync(dev + s0, pin, fill, hipMemcpyHostToDevice, c->copy));
        CK(c, hipEventRecord(c->pin_ev[ps], c->copy));
        c->pin_used[ps] = true;
        k = k1;
    }
    c->st.h2d_ms_total += now_ms() - t0;
    c->st.h2d_bytes_total += m.bytes;
    c->st.h2d_staged_bytes_total += m.bytes;
    return PGH_OK;
}

// pgh_ingest_state of a page-locked message: [first payload, last payload end) of this shard in one
// DMA to d_vbytes, the gather table behind it, then k_gather_f32 into the slot's row.  `ranged`
// (pgh_set_ingest_ranges): the table's chunks are cut at INGEST_CHUNK param boundaries and the DMA +
// gather run chunk by chunk, rng_ev[k] behind chunk k's gather.
int pinned_gather_ingest(pgh_ctx* c, const uint8_t* pb, const std::vector<Piece>& pieces, int slot, bool ranged) {
    const size_t a = (size_t)(pieces.front().src - pb) & ~(size_t)63;
    const size_t b = (size_t)(pieces.back().src - pb) + pieces.back().n;
    std::vector<pgh::GChunk> tab;
    int64_t dst = 0;
    size_t total = 0;
    for (auto& p : pieces) {
        const int64_t nf = (int64_t)(p.n / 4);
        const int64_t src = (int64_t)((size_t)(p.src - pb) - a);
        for (int64_t k = 0; k < nf;) {
            int64_t len = std::min<int64_t>(pgh::GATHER_CHUNK, nf - k);
            if (ranged) len = std::min(len, (((dst + k) / INGEST_CHUNK) + 1) * INGEST_CHUNK - (dst + k));
            tab.push_back({src + 4 * k, dst + k, (int32_t)len, 0});
            k += len;
        }
        dst += nf;
        total += p.n;
    }
    ranged = ranged && dst == c->pg;
    if (tab.empty()) return PGH_OK;
    RC(grow_device(c, (void**)&c->d_vbytes, &c->vbytes_cap, b - a + 16, "pinned message buffer"));
    const size_t tb = tab.size() * sizeof(pgh::GChunk);
    if (!c->gtab_ev) CK(c, hipEventCreateWithFlags(&c->gtab_ev, hipEventDisableTiming));
    if (!c->gdma_ev) CK(c, hipEventCreateWithFlags(&c->gdma_ev, hipEventDisableTiming));
    if (c->gtab_used) CK(c, hipEventSynchronize(c->gtab_ev));  // the previous table upload read h_gtab
    if (tb > c->gtab_cap) {
        if (c->h_gtab) (void)hipHostFree(c->h_gtab);
        c->h_gtab = nullptr;
        size_t cap = 0;
        void* d = c->d_gtab;
        RC(grow_device(c, &d, &cap, tb, "gather chunk table"));
        c->d_gtab = (pgh::GChunk*)d;
        if (hipHostMalloc((void**)&c->h_gtab, cap, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            c->gtab_cap = 0;
            return fail(c, PGH_E_OOM, "pinned gather table of %zu bytes failed", cap);
        }
        c->gtab_cap = cap;
        c->gtab_used = false;
    }
    std::memcpy(c->h_gtab, tab.data(), tb);
    ++c->copy_seq;
    CK(c, hipMemcpyAsync(c->d_gtab, c->h_gtab, tb, hipMemcpyHostToDevice, c->copy));
    CK(c, hipEventRecord(c->gtab_ev, c->copy));
    c->gtab_used = true;
    const Dest d = row_dest(c, slot, 0);
    const bool async = host_async(pb + a, b - a);
    if (ranged) {
        const int K = (int)((c->pg + INGEST_CHUNK - 1) / INGEST_CHUNK);
        while ((int)c->rng_ev.size() < K) {
            hipEvent_t ev = nullptr;
            CK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            c->rng_ev.push_back(ev);
        }
        size_t e0 = 0;
        for (int k = 0; k < K; ++k) {
            size_t e1 = e0;
            while (e1 < tab.size() && tab[e1].dst < (int64_t)(k + 1) * INGEST_CHUNK) ++e1;
            if (e1 > e0) {
                const size_t lo = (size_t)tab[e0].src, hi = (size_t)tab[e1 - 1].src + 4 * (size_t)tab[e1 - 1].n;
                CK(c, hipMemcpyAsync(c->d_vbytes + lo, pb + a + lo, hi - lo, hipMemcpyHostToDevice, c->copy));
                if (e1 == tab.size()) {  // the message's last DMA: the host block is read once this is done
                    if (async) RC(host_dma_queued(c, pb + a, b - a, c->copy));
                    else CK(c, hipEventRecord(c->gdma_ev, c->copy));
                }
                const hipError_t e = pgh::launch_gather_f32(c->d_vbytes, c->d_gtab + e0, (int)(e1 - e0),
                                                            (float*)d.base, d.map, c->copy);
                if (e != hipSuccess) return fail(c, PGH_E_HIP, "gather launch failed: %s", hipGetErrorString(e));
            }
            CK(c, hipEventRecord(c->rng_ev[(size_t)k], c->copy));
            e0 = e1;
        }
        c->rng_seq = c->copy_seq;
        c->rng_n = K;
    } else {
        CK(c, hipMemcpyAsync(c->d_vbytes, pb + a, b - a, hipMemcpyHostToDevice, c->copy));
        if (async) RC(host_dma_queued(c, pb + a, b - a, c->copy));  // the block's owner waits (pgh_host_wait)
        else CK(c, hipEventRecord(c->gdma_ev, c->copy));
        const hipError_t e = pgh::launch_gather_f32(c->d_vbytes, c->d_gtab, (int)tab.size(), (float*)d.base, d.map,
                                                    c->copy);
        if (e != hipSuccess) return fail(c, PGH_E_HIP, "gather launch failed: %s", hipGetErrorString(e));
    }
    if (!async) CK(c, hipEventSynchronize(c->gdma_ev));
    c->st.h2d_bytes_total += total;
    return PGH_OK;
}

// A varint buffer holding `bytes` of messages and a table of `tab_bytes` (grown when short, after
// the decode that last read it).  The dec stream and its events are made on the first use.
int prepare_vbuf(pgh_ctx* c, pgh_ctx::VarintBuf& b, size_t bytes, size_t tab_bytes) {
    if (!c->dec) {
        CK(c, hipStreamCreateWithFlags(&c->dec, hipStreamNonBlocking));
        CK(c, hipEventCreateWithFlags(&c->dec_in, hipEventDisableTiming));
        for (auto& x : c->vbuf) CK(c, hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
    }
    if ((bytes > b.cap || tab_bytes > b.tab_cap) && b.used) CK(c, hipEventSynchronize(b.done));
    RC(grow_device(c, (void**)&b.bytes, &b.cap, bytes, "share payload buffer"));
    void* t = b.tab;
    RC(grow_device(c, &t, &b.tab_cap, tab_bytes, "varint chunk table"));
    b.tab = (pgh::VChunk*)t;
    // the copy stream's DMAs into this buffer wait for the decode that last read it (two messages ago)
    if (b.used) CK(c, hipStreamWaitEvent(c->copy, b.done, 0));
    return PGH_OK;
}

// Every party validated: one chunk table for all of them (uploaded behind the payload DMAs), then
// one decode per party into its slab row (the shard's range), on the dec stream.
int decode_share_msgs(pgh_ctx* c, std::vector<ShareMsg>& msgs, int slot, pgh_ctx::VarintBuf& b) {
    size_t nk = 0;
    for (auto& m : msgs) nk += m.chunks.size();
    if (nk == 0) return PGH_OK;  // every tensor empty
    const size_t tb = nk * sizeof(pgh::VChunk);
    if (!c->vtab_ev) CK(c, hipEventCreateWithFlags(&c->vtab_ev, hipEventDisableTiming));
    if (c->vtab_used) CK(c, hipEventSynchronize(c->vtab_ev));  // the previous table upload read h_vtab
    if (tb > c->vtab_cap) {
        if (c->h_vtab) (void)hipHostFree(c->h_vtab);
        c->h_vtab = nullptr;
        c->vtab_cap = 0;
        if (hipHostMalloc((void**)&c->h_vtab, b.tab_cap, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            c->h_vtab = nullptr;
            return fail(c, PGH_E_OOM, "pinned chunk table of %zu bytes failed", b.tab_cap);
        }
        c->vtab_cap = b.tab_cap;
        c->vtab_used = false;
    }
    size_t at = 0;
    for (auto& m : msgs) {
        std::memcpy(c->h_vtab + at, m.chunks.data(), m.chunks.size() * sizeof(pgh::VChunk));
        at += m.chunks.size();
    }
    ++c->copy_seq;
    CK(c, hipMemcpyAsync(b.tab, c->h_vtab, tb, hipMemcpyHostToDevice, c->copy));
    CK(c, hipEventRecord(c->vtab_ev, c->copy));
    c->vtab_used = true;
    CK(c, hipEventRecord(c->dec_in, c->copy));
    CK(c, hipStreamWaitEvent(c->dec, c->dec_in, 0));
    at = 0;
    for (size_t s = 0; s < msgs.size(); ++s) {
        const int n = (int)msgs[s].chunks.size();
        const hipError_t e = pgh::launch_varint_decode(b.bytes, b.tab + at, n, (int64_t*)slot_row(c, slot, (int)s),
                                                       slab_map(c), c->lo, c->hi, c->dec);
        if (e != hipSuccess) return fail(c, PGH_E_HIP, "varint decode launch failed: %s", hipGetErrorString(e));
        at += (size_t)n;
    }
    CK(c, hipEventRecord(b.done, c->dec));
    b.used = true;
    c->dec_last = b.done;
    return PGH_OK;
}
}  // namespace

int pgh_ingest_state_shares(pgh_ctx* c, int client, int n_parties, const uint8_t* const* pbs, const size_t* ns) {
    if (c && c->grp) return pgh_group_api::ingest_state_shares(c, client, n_parties, pbs, ns);
    RC(check_dtype(c, PGH_I64));
    if (!pbs || !ns) return fail(c, PGH_E_ARG, "pbs / ns is NULL");
    if (n_parties != c->parties)
        return fail(c, PGH_E_ARG, "client %d: %d share messages, context holds %d parties", client, n_parties,
                    c->parties);
    // all parties are staged and validated before any is decoded: a bad message leaves the slab as it was
    std::vector<ShareMsg> msgs((size_t)n_parties);
    size_t total = 0;
    for (int s = 0; s < n_parties; ++s) {
        if (!pbs[s] && ns[s]) return fail(c, PGH_E_ARG, "client %d party %d: NULL message", client, s);
        total = (total + 15) & ~(size_t)15;
        RC(plan_share_msg(c, pbs[s], ns[s], client, s, total, &msgs[(size_t)s]));
        total += msgs[(size_t)s].bytes;
    }
    size_t nk = 0;
    for (auto& m : msgs) nk += m.chunks.size();
    DeviceGuard g(c->device);
    int slot = 0;
    RC(claim_slot(c, client, &slot));
    pgh_ctx::VarintBuf& b = c->vbuf[c->vbuf_next];
    c->vbuf_next ^= 1;
    RC(prepare_vbuf(c, b, total + 16, std::max<size_t>(nk, 1) * sizeof(pgh::VChunk)));
    for (auto& m : msgs) RC(stage_share_msg(c, m, b.bytes));
    for (int s = 0; s < n_parties; ++s) RC(check_share_msg(c, &msgs[(size_t)s], client, s));
    RC(decode_share_msgs(c, msgs, slot, b));
    return mark_ingested(c, client, slot);
}

int pgh_synth_ingest(pgh_ctx* c, uint64_t seed, int client0, int n) {
    if (c && c->grp) return pgh_group_api::synth_ingest(c, seed, client0, n);
    RC(check_ready(c));
    if (n <= 0 || client0 < 0) return fail(c, PGH_E_ARG, "bad client range %d + %d", client0, n);
    DeviceGuard g(c->device);
    int k = 0;
    while (k < n) {
        const int64_t client = (int64_t)client0 + k;
        int slot = 0;
        RC(claim_slot(c, client, &slot));
        // contiguous run of slots from `slot`, all claimable
        int run = 1;
        while (k + run < n && slot + run < c->slots && run < 65535) {  // 65535: synth grid rows
            const int64_t cl = client + run;
            if (c->streaming) {
                const int64_t held = c->slot_client[(size_t)(slot + run)];
                if (held >= 0 && held != cl) break;
            } else if (cl >= c->slots) {
                break;
            }
            ++run;
        }
        if (c->streaming && run > 1) RC(order_stream_overwrite(c, client + run - 1));
        hipError_t e;
        // STREAM fills run on the fold stream, generator and fold alternating with the whole GPU each
        // (beside the fold on the copy stream, the write-heavy fill and the read-only fold shared
        // HBM 13 % worse, r02p), grid capped at 8192 workgroups (r01t), non-temporal stores
        const hipStream_t gs = c->streaming ? c->stream : c->copy;
        ++c->copy_seq;
        if (c->dtype == PGH_F32)
            e = pgh::launch_synth_f32((float*)slot_row(c, slot, 0), slab_map(c), c->nb * c->bw, run, c->pg, seed,
                                      pgh::STREAM_DIFF, c->client_base + client, c->lo, pgh::DIFF_SCALE, gs,
                                      c->streaming ? 8192 : 0, c->synth_kind, true);
        else
            e = pgh::launch_synth_shares((int64_t*)slot_row(c, slot, 0), slab_map(c), c->nb * c->bw, run, c->parties,
                                         c->pg, seed, c->client_base + client, c->lo, 1000.0f, gs);
        if (e != hipSuccess) return fail(c, PGH_E_HIP, "synthetic fill failed: %s", hipGetErrorString(e));
        for (int j = 0; j < run; ++j) {
            if (c->slot_client[(size_t)(slot + j)] != client + j) c->st.n_clients += 1;
            c->slot_client[(size_t)(slot + j)] = client + j;
        }
        if (c->streaming) RC(maybe_fold(c, false));
        k += run;
    }
    return PGH_OK;
}

int pgh_set_synth_kind(pgh_ctx* c, int kind) {
    if (c && c->grp) return pgh_group_api::set_synth_kind(c, kind);
    if (!c) return PGH_E_ARG;
    if (kind != 0 && kind != 1) return fail(c, PGH_E_ARG, "synthetic generator kind %d is not 0 or 1", kind);
    c->synth_kind = kind;
    return PGH_OK;
}

int pgh_set_ingest_ranges(pgh_ctx* c, int on) {
    if (c && c->grp) return pgh_group_api::set_ingest_ranges(c, on);
    if (!c) return PGH_E_ARG;
    c->ingest_ranges = on != 0;
    return PGH_OK;
}

int pgh_synth_fill(pgh_ctx* c, uint64_t seed, int n_clients) {
    if (c && c->grp) return pgh_group_api::synth_fill(c, seed, n_clients);
    RC(check_ready(c));
    if (c->streaming) return fail(c, PGH_E_STATE, "pgh_synth_fill is for resident slabs; use pgh_synth_ingest");
    if (n_clients <= 0 || n_clients > c->slots)
        return fail(c, PGH_E_ARG, "n_clients %d outside (0,%d]", n_clients, c->slots);
    RC(pgh_reset(c));
    return pgh_synth_ingest(c, seed, 0, n_clients);
}

int pgh_synth_ckpt_device(pgh_ctx* c, uint64_t seed, float* d_ckpt, void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (!d_ckpt || ((uintptr_t)d_ckpt & 15)) return fail(c, PGH_E_ARG, "d_ckpt must be a 16-byte aligned device pointer");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    if (c->pg % 4 == 0) {  // one row of exactly P_shard elements
        hipError_t e = pgh::launch_synth_f32(d_ckpt, pgh::single_block(c->pg), c->pg, 1, c->pg, seed, pgh::STREAM_CKPT, 0,
                                             c->lo, pgh::CKPT_SCALE, s);
        if (e != hipSuccess) return fail(c, PGH_E_HIP, "synthetic checkpoint failed: %s", hipGetErrorString(e));
        return PGH_OK;
    }
    if (!c->d_ckpt) return fail(c, PGH_E_STATE, "pgh_reserve has not been called");
    c->ckpt_valid = false;  // the resident checkpoint is used as scratch here
    clear_final_marks(c);
    hipError_t e = pgh::launch_synth_f32(c->d_ckpt, pgh::single_block(c->pvec), c->pvec, 1, c->pg, seed,
                                         pgh::STREAM_CKPT, 0, c->lo, pgh::CKPT_SCALE, s);
    if (e != hipSuccess) return fail(c, PGH_E_HIP, "synthetic checkpoint failed: %s", hipGetErrorString(e));
    CK(c, hipMemcpyAsync(d_ckpt, c->d_ckpt, sizeof(float) * c->pg, hipMemcpyDeviceToDevice, s));
    return PGH_OK;
}

int pgh_set_weights(pgh_ctx* c, const float* w, int n) {
    if (c && c->grp) return pgh_group_api::set_weights(c, w, n);
    if (!c) return PGH_E_ARG;
    if (!w || n <= 0) return fail(c, PGH_E_ARG, "need a non-empty weight vector");
    if (c->folded > 0) {  // stream or slot folds: clients [0, folded) are in the running state
        for (int64_t k = 0; k < c->folded && k < n && k < (int64_t)c->weights.size(); ++k)
            if (std::memcmp(&w[k], &c->weights[(size_t)k], 4) != 0)
                return fail(c, PGH_E_STATE, "weight of already folded client %lld changed", (long long)k);
        if (n < c->folded) return fail(c, PGH_E_STATE, "fewer weights than folded clients");
    }
    c->weights.assign(w, w + n);
    c->weights_on_device = false;
    return PGH_OK;
}

