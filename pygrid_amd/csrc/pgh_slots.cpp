// libpygrid_hip: report-time folds of scattered slots -- the certain prefix of the close-time order
// folded as its diffs arrive, in any slot.  Reference: submit_worker_diff (cycle_manager.py:151-178)
// feeding _average_plan_diffs (:219-323).  (struct pgh_ctx and the shared helpers: pgh_ctx.h)
#include "pgh_ctx.h"

using namespace pgh_detail;

// (the public entry points take their C linkage from include/pgh_api.h)

// ---- report-time folds of scattered slots (pgh_fold_slots) -------------------------------------

namespace {
int slot_fold(pgh_ctx* c, int mode, const int32_t* slots, int n, bool final) {
    RC(check_dtype(c, PGH_F32));
    if (!valid_mode(mode)) return fail(c, PGH_E_ARG, "unknown averaging mode %d", mode);
    if (c->streaming) return fail(c, PGH_E_STATE, "context is streaming: slot folds need a RESIDENT slab");
    if (n < 0 || (n > 0 && !slots)) return fail(c, PGH_E_ARG, "bad slot list (n=%d)", n);
    if (c->slot_mode >= 0 && c->slot_mode != mode)
        return fail(c, PGH_E_STATE, "averaging mode changed from %d to %d within a cycle", c->slot_mode, mode);
    std::vector<char> seen((size_t)c->slots, 0);
    for (int k = 0; k < n; ++k) {
        const int32_t sl = slots[k];
        if (sl < 0 || sl >= c->slots) return fail(c, PGH_E_ARG, "slot %d outside [0,%d)", sl, c->slots);
        if (c->slot_client[(size_t)sl] < 0) return fail(c, PGH_E_STATE, "slot %d holds no unfolded diff", sl);
        if (seen[(size_t)sl]) return fail(c, PGH_E_ARG, "slot %d listed twice", sl);
        seen[(size_t)sl] = 1;
    }
    const int64_t c0 = c->folded, total = c0 + n;
    FinalArgs fa;
    if (final) {
        RC(check_ckpt(c, "pgh_fold_slots_finish_resident"));
        if (total == 0) return fail(c, PGH_E_STATE, "no diffs folded");
        RC(fedavg_divisor(c, mode, total, &fa.divisor));
    } else if (n == 0) {
        return PGH_OK;
    }
    DeviceGuard g(c->device);
    const hipStream_t s = c->stream;
    // a close right behind a ranged ingest (pgh_set_ingest_ranges) orders each FINAL range after the
    // chunk of the last report it reads instead of after the whole copy stream
    const bool ranged = final && n > 0 && n <= pgh::ROWTAB_MAX && c->pg >= (1 << 20) && ranged_ingest_valid(c);
    if (!ranged) RC(order_after_ingest(c, s));
    else if (c->dec_last) CK(c, hipStreamWaitEvent(s, c->dec_last, 0));  // the copy stream: per range below
    if (mode == PGH_WEIGHTED_MEAN && n > 0) {
        if ((int64_t)c->weights.size() < total)
            return fail(c, PGH_E_STATE, "weighted mean: %zu weights for %lld clients", c->weights.size(),
                        (long long)total);
        RC(sync_weights(c, s));
    }
    if (mode == PGH_ITERATIVE_MEAN && n > 0) RC(ensure_recips(c, total, s));
    int done = 0;
    bool prequeued = false;
    do {
        const int m = std::min(n - done, pgh::ROWTAB_MAX);
        pgh::RowTab tab;
        for (int k = 0; k < m; ++k) tab.rows[k] = slots[done + k] * c->parties;
        const bool first = (c0 + done == 0), last = (done + m == n);
        pgh::FedavgArgs a{};
        a.diffs = (const float*)c->d_slab;
        a.map = slab_map(c);
        a.n_rows = m;
        a.client0 = c0 + done;
        a.p = c->pg;
        a.weights = c->d_w ? c->d_w + (c0 + done) : nullptr;
        a.recips = c->d_rec ? c->d_rec + (c0 + done) : nullptr;
        a.acc = c->d_acc;
        a.ckpt = c->d_ckpt;
        a.out = c->d_out;
        a.divisor = fa.divisor;
        a.flags = (first ? pgh::FL_FIRST : 0) | (final && last ? pgh::FL_FINAL : 0);
        a.mode = mode;
        a.variant = c->variant;
        // The FINAL pass of a report-time close (a short fold of the rows left) as ranges of 4 MiB of
        // output, one after another on one stream, a mark behind every second one: each 8 MiB D2H
        // piece starts behind the two ranges that wrote it instead of behind the whole fold.  Ranges
        // aligned to the pieces on one stream closed 0.1-0.15 ms sooner than 8 equal ranges
        // alternating over two streams (profiles/r04m/: 2.04 vs 2.19 ms, close start -> new
        // checkpoint bytes); a mark (a system-scope release) only where a piece ends (r05).
        const int64_t RF = (int64_t)(D2H_PIECE / 8);
        const int K = (a.flags & pgh::FL_FINAL) && c->pg >= (1 << 20) ? (int)((c->pg + RF - 1) / RF) : 1;
        if (a.flags & pgh::FL_FINAL) clear_final_marks(c);
        // the new checkpoint's D2H starts here: after each mark, the pieces whose ranges have
        // finished go out while the later ranges are still being issued (stage_d2h_pieces adopts the
        // ring).  The result is d_out until the swap below.
        pgh_ctx::D2HRing& pre = c->pre_d2h;
        bool prequeue = false;
        if (K > 1 && (a.flags & pgh::FL_FINAL)) {
            RC(d2h_ring_begin(c, &pre, (const uint8_t*)c->d_out, 4 * (size_t)c->pg, s, true, false));
            prequeue = pre.base || pre.n_free > 0;  // own cells, or a free staging slot
        }
        for (int r = 0; r < K; ++r) {
            const hipStream_t rs = s;
            const int64_t lo = std::min(c->pg, RF * r), hi = K == 1 ? c->pg : std::min(c->pg, RF * (r + 1));
            if (ranged && K > 1) {  // every chunk this range reads has landed ...
                for (int64_t k = lo / INGEST_CHUNK; k <= (hi - 1) / INGEST_CHUNK; ++k)
                    CK(c, hipStreamWaitEvent(rs, c->rng_ev[(size_t)k], 0));
            } else if (ranged && r == 0) {
                CK(c, hipStreamWaitEvent(rs, c->rng_ev[(size_t)(c->rng_n - 1)], 0));  // ... or all of it
            }
            pgh::FedavgArgs ar = a;
            ar.map.off = lo;
            ar.p = hi - lo;
            ar.acc = c->d_acc + lo;
            ar.ckpt = c->d_ckpt + lo;
            ar.out = c->d_out + lo;
            const uint64_t rp = (uint64_t)(hi - lo);
            const uint64_t bytes = 4ull * (uint64_t)m * rp + (first ? 0 : 4 * rp) + ((a.flags & pgh::FL_FINAL) ? 8 * rp : 4 * rp);
            RC(timed_launch(c, rs, bytes, [&] { return pgh::launch_fedavg_rows(ar, tab, rs); }));
            if (K > 1 && (hi % (2 * RF) == 0 || hi == c->pg)) {
                RC(add_final_mark(c, rs, hi));
                const size_t before = prequeue ? pre.queued : 0;
                if (prequeue) RC(d2h_issue_ready(c, &pre));
                if (prequeue && pre.queued > before)  // its slots are busy until these pieces land
                    for (int k = 0; k < pre.n_free; ++k) {
                        CK(c, hipEventRecord(c->pin_ev[pre.free_slot[k]], pre.s));
                        c->pin_used[pre.free_slot[k]] = true;
                    }
            }
        }
        prequeued = prequeued || prequeue;
        done += m;
    } while (done < n);
    RC(record_fold(c, s));
    RC(record_slot_fold(c, slots, n));
    for (int k = 0; k < n; ++k) c->slot_client[(size_t)slots[k]] = -1;  // free for the next ingests
    c->folded = total;
    c->st.n_folded = total;
    c->slot_mode = mode;
    if (final) {
        std::swap(c->d_ckpt, c->d_out);  // the new checkpoint is the next cycle's input
        c->pre_d2h_valid = prequeued && c->pre_d2h.src == (const uint8_t*)c->d_ckpt;
        c->folded = 0;  // the next cycle folds from scratch
        c->slot_mode = -1;
    }
    return PGH_OK;
}
}  // namespace

int pgh_fold_slots(pgh_ctx* c, int mode, const int32_t* slots, int n) {
    if (c && c->grp) return pgh_group_api::fold_slots(c, mode, slots, n, false);
    if (!c) return PGH_E_ARG;
    return slot_fold(c, mode, slots, n, false);
}

int pgh_fold_slots_finish_resident(pgh_ctx* c, int mode, const int32_t* slots, int n) {
    if (c && c->grp) return pgh_group_api::fold_slots(c, mode, slots, n, true);
    if (!c) return PGH_E_ARG;
    const double t0 = now_ms();
    RC(slot_fold(c, mode, slots, n, true));
    c->st.close_ms_last = now_ms() - t0;
    return PGH_OK;
}

namespace {
int check_slot_folds(pgh_ctx* c) {
    RC(check_dtype(c, PGH_F32));
    if (c->streaming) return fail(c, PGH_E_STATE, "context is streaming: slot folds need a RESIDENT slab");
    return PGH_OK;
}
}  // namespace

int pgh_fold_slots_restart(pgh_ctx* c) {
    if (c && c->grp) return pgh_group_api::fold_restart(c);
    if (!c) return PGH_E_ARG;
    RC(check_slot_folds(c));
    // The next slot fold's FL_FIRST pass overwrites the fold state on c->stream, behind any fold
    // still in flight there: nothing to wait for.
    c->folded = 0;
    c->st.n_folded = 0;
    c->slot_mode = -1;
    c->weights.clear();
    c->weights_on_device = false;
    return PGH_OK;
}
