// libpygrid_hip: report-time folds of scattered slots (every reported diff folded as it arrives,
// any order), saved fold states (mark / rewind / unmark) and the speculative close (pgh_fold_peek*:
// the FINAL pass, its D2H and the payload copy-out taken ahead of the close).  Reference:
// submit_worker_diff (cycle_manager.py:151-178) feeding _average_plan_diffs (:219-323).
// (struct pgh_ctx and the shared helpers: pgh_ctx.h)
#include "pgh_ctx.h"

using namespace pgh_detail;

namespace pgh_detail {

// Wait until the peek thread is idle (its copy read h_peek and wrote the caller's buffer).
void peek_job_wait(pgh_ctx* c) {
    std::unique_lock<std::mutex> lk(c->pk_mu);
    c->pk_cv.wait(lk, [c] { return !c->pk_busy; });
}

void peek_thread_stop(pgh_ctx* c) {
    if (!c->pk_thread.joinable()) return;
    {
        std::lock_guard<std::mutex> lk(c->pk_mu);
        c->pk_stop = true;
    }
    c->pk_cv.notify_all();
    c->pk_thread.join();
}

}  // namespace pgh_detail

namespace {

void peek_thread_main(pgh_ctx* c) {
    (void)hipSetDevice(c->device);
    for (;;) {
        uint8_t* out = nullptr;
        std::vector<std::pair<uint8_t*, size_t>> pieces;
        uint64_t gen = 0;
        {
            std::unique_lock<std::mutex> lk(c->pk_mu);
            c->pk_cv.wait(lk, [c] { return c->pk_stop || (c->pk_busy && c->pk_out); });
            if (c->pk_stop) return;
            out = c->pk_out;
            pieces.swap(c->pk_pieces);
            gen = c->pk_gen;
        }
        // piece k of the D2H (D2H_PIECE bytes of h_peek) is copied out as soon as its event fires
        std::vector<OutPiece> op;
        size_t total = 0;
        for (auto& pc : pieces) {
            op.push_back(OutPiece{pc.first, pc.second});
            total += pc.second;
        }
        bool ok = true;
        for (size_t k = 0; ok && k < c->peek_pieces && k * D2H_PIECE < total; ++k) {
            ok = hipEventSynchronize(c->peek_piece_ev[k]) == hipSuccess;
            const size_t off = k * D2H_PIECE, len = std::min(D2H_PIECE, total - off);
            if (ok) scatter_out((const uint8_t*)c->h_peek + off, off, len, op, *c->pool_peek);
        }
        ok = ok && hipEventSynchronize(c->peek_ev) == hipSuccess;
        {
            std::lock_guard<std::mutex> lk(c->pk_mu);
            c->pk_done_gen = ok ? gen : 0;
            c->pk_done_out = out;
            c->pk_out = nullptr;
            c->pk_busy = false;
        }
        c->pk_cv.notify_all();
    }
}

}  // namespace

// (the public entry points take their C linkage from include/pgh_api.h)

// ---- report-time folds of scattered slots (pgh_fold_slots) -------------------------------------

namespace {
int slot_fold(pgh_ctx* c, int mode, const int32_t* slots, int n, bool final, bool keep = false) {
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
    RC(order_after_ingest(c, s));
    if (mode == PGH_WEIGHTED_MEAN && n > 0) {
        if ((int64_t)c->weights.size() < total)
            return fail(c, PGH_E_STATE, "weighted mean: %zu weights for %lld clients", c->weights.size(),
                        (long long)total);
        RC(sync_weights(c, s));
    }
    if (mode == PGH_ITERATIVE_MEAN && n > 0) RC(ensure_recips(c, total, s));
    int done = 0;
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
        // output, one after another on one stream, each followed by its mark: the D2H pieces (8 MiB)
        // start behind the first two instead of behind the whole fold.  Ranges aligned to the pieces on
        // one stream closed 0.1-0.15 ms sooner than 8 equal ranges alternating over two streams
        // (profiles/r04m/: 2.04 vs 2.19 ms, close start -> new checkpoint bytes).
        const int64_t RF = (int64_t)(D2H_PIECE / 8);
        const int K = (a.flags & pgh::FL_FINAL) && c->pg >= (1 << 20) ? (int)((c->pg + RF - 1) / RF) : 1;
        if (a.flags & pgh::FL_FINAL) clear_final_marks(c);
        for (int r = 0; r < K; ++r) {
            const hipStream_t rs = s;
            const int64_t lo = std::min(c->pg, RF * r), hi = K == 1 ? c->pg : std::min(c->pg, RF * (r + 1));
            pgh::FedavgArgs ar = a;
            ar.map.off = lo;
            ar.p = hi - lo;
            ar.acc = c->d_acc + lo;
            ar.acc_in = (done == 0 && c->acc_src) ? c->acc_src + lo : nullptr;  // rewound: the mark's buffer
            ar.ckpt = c->d_ckpt + lo;
            ar.out = c->d_out + lo;
            const uint64_t rp = (uint64_t)(hi - lo);
            const uint64_t bytes = 4ull * (uint64_t)m * rp + (first ? 0 : 4 * rp) + ((a.flags & pgh::FL_FINAL) ? 8 * rp : 4 * rp);
            RC(timed_launch(c, rs, bytes, [&] { return pgh::launch_fedavg_rows(ar, tab, rs); }));
            if (K > 1) RC(add_final_mark(c, rs, hi));
        }
        done += m;
    } while (done < n);
    RC(record_fold(c, s));
    RC(record_slot_fold(c, slots, n));
    ++c->state_gen;
    c->acc_src = nullptr;  // the running state is in d_acc again
    if (!keep)
        for (int k = 0; k < n; ++k) c->slot_client[(size_t)slots[k]] = -1;  // free for the next ingests
    c->folded = total;
    c->st.n_folded = total;
    c->slot_mode = mode;
    if (final) {
        std::swap(c->d_ckpt, c->d_out);  // the new checkpoint is the next cycle's input
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

int pgh_fold_slots_keep(pgh_ctx* c, int mode, const int32_t* slots, int n) {
    if (c && c->grp) return pgh_group_api::fold_slots_keep(c, mode, slots, n);
    if (!c) return PGH_E_ARG;
    return slot_fold(c, mode, slots, n, false, true);
}

namespace {
int check_slot_folds(pgh_ctx* c) {
    RC(check_dtype(c, PGH_F32));
    if (c->streaming) return fail(c, PGH_E_STATE, "context is streaming: slot folds need a RESIDENT slab");
    return PGH_OK;
}
constexpr size_t MAX_FOLD_MARKS = 4096;
}  // namespace

int pgh_fold_mark(pgh_ctx* c, int mark) {
    if (c && c->grp) return pgh_group_api::fold_mark(c, mark);
    if (!c) return PGH_E_ARG;
    RC(check_slot_folds(c));
    if (mark < 0) return fail(c, PGH_E_ARG, "negative mark %d", mark);
    auto it = c->fold_marks.find(mark);
    if (it == c->fold_marks.end() && c->fold_marks.size() >= MAX_FOLD_MARKS)
        return fail(c, PGH_E_STATE, "more than %zu saved fold states", MAX_FOLD_MARKS);
    DeviceGuard g(c->device);
    pgh_ctx::SavedFold m{nullptr, c->folded, c->slot_mode};
    if (c->folded > 0) {
        float* spare = nullptr;
        if (!c->acc_spare.empty()) {
            spare = c->acc_spare.back();
            c->acc_spare.pop_back();
        } else if (hipMalloc((void**)&spare, (size_t)c->pvec * 4) != hipSuccess) {
            (void)hipGetLastError();
            return fail(c, PGH_E_OOM, "fold state buffer (%lld floats) allocation failed", (long long)c->pvec);
        }
        if (c->acc_src) {
            // right after a rewind the state lives in another mark's buffer: this mark gets a copy
            CK(c, hipMemcpyAsync(spare, c->acc_src, (size_t)c->pg * 4, hipMemcpyDeviceToDevice, c->stream));
            m.buf = spare;
        } else {
            // the mark keeps d_acc as it stands; the next fold reads it there and writes the spare
            m.buf = c->d_acc;
            c->d_acc = spare;
            c->acc_src = m.buf;
        }
    }
    if (it != c->fold_marks.end()) {
        if (it->second.buf) {
            if (c->acc_src == it->second.buf) {  // the pending state is the mark being replaced
                CK(c, hipMemcpyAsync(c->d_acc, c->acc_src, (size_t)c->pg * 4, hipMemcpyDeviceToDevice, c->stream));
                c->acc_src = nullptr;
            }
            c->acc_spare.push_back(it->second.buf);
        }
        it->second = m;
    } else {
        c->fold_marks.emplace(mark, m);
    }
    return PGH_OK;
}

int pgh_fold_rewind(pgh_ctx* c, int mark) {
    if (c && c->grp) return pgh_group_api::fold_rewind(c, mark);
    if (!c) return PGH_E_ARG;
    RC(check_slot_folds(c));
    auto it = c->fold_marks.find(mark);
    if (it == c->fold_marks.end()) return fail(c, PGH_E_ARG, "no saved fold state %d", mark);
    c->folded = it->second.folded;
    c->st.n_folded = c->folded;
    c->slot_mode = it->second.folded > 0 ? it->second.mode : -1;
    c->acc_src = it->second.buf;  // the next slot fold reads the state there (no copy)
    ++c->state_gen;
    return PGH_OK;
}

int pgh_fold_unmark(pgh_ctx* c, int mark) {
    if (c && c->grp) return pgh_group_api::fold_unmark(c, mark);
    if (!c) return PGH_E_ARG;
    RC(check_slot_folds(c));
    auto it = c->fold_marks.find(mark);
    if (it == c->fold_marks.end()) return fail(c, PGH_E_ARG, "no saved fold state %d", mark);
    if (it->second.buf) {
        if (c->acc_src == it->second.buf) {  // rewound to it and not folded since: keep the state
            DeviceGuard g(c->device);
            CK(c, hipMemcpyAsync(c->d_acc, c->acc_src, (size_t)c->pg * 4, hipMemcpyDeviceToDevice, c->stream));
            c->acc_src = nullptr;
        }
        c->acc_spare.push_back(it->second.buf);
    }
    c->fold_marks.erase(it);
    return PGH_OK;
}

// ---- speculative close: the FINAL pass of the fold state as it stands, ahead of the close -----------

int pgh_fold_peek(pgh_ctx* c, int mode) {
    if (c && c->grp) return pgh_group_api::fold_peek(c, mode);
    if (!c) return PGH_E_ARG;
    RC(check_slot_folds(c));
    RC(check_ckpt(c, "pgh_fold_peek"));
    if (!valid_mode(mode)) return fail(c, PGH_E_ARG, "unknown averaging mode %d", mode);
    if (c->folded <= 0) return fail(c, PGH_E_STATE, "pgh_fold_peek: nothing folded yet");
    if (c->slot_mode >= 0 && c->slot_mode != mode)
        return fail(c, PGH_E_STATE, "averaging mode changed from %d to %d within a cycle", c->slot_mode, mode);
    FinalArgs fa;
    RC(fedavg_divisor(c, mode, c->folded, &fa.divisor));
    DeviceGuard g(c->device);
    if (c->peek_stream) {
        // the previous peek's copy still running (reports arriving faster than 47 MB cross PCIe):
        // skip this one rather than stall the fold stream behind it -- the close then folds itself
        const hipError_t q = hipEventQuery(c->peek_ev);
        bool busy = q == hipErrorNotReady;
        if (busy) (void)hipGetLastError();
        {
            std::lock_guard<std::mutex> lk(c->pk_mu);
            busy = busy || c->pk_busy;
        }
        if (busy) {
            c->peek_gen = 0;
            return PGH_OK;
        }
        if (q != hipSuccess) return fail(c, PGH_E_HIP, "hipEventQuery failed: %s", hipGetErrorString(q));
    }
    if (!c->peek_stream) {
        CK(c, hipStreamCreateWithFlags(&c->peek_stream, hipStreamNonBlocking));
        CK(c, hipEventCreateWithFlags(&c->peek_ev, hipEventDisableTiming));
    }
    if (!c->d_peek && hipMalloc((void**)&c->d_peek, (size_t)c->pvec * 4) != hipSuccess) {
        (void)hipGetLastError();
        c->d_peek = nullptr;
        return fail(c, PGH_E_OOM, "peek buffer (%lld floats) allocation failed", (long long)c->pvec);
    }
    if (c->peek_cap < (size_t)c->pg) {
        CK(c, hipStreamSynchronize(c->peek_stream));
        if (c->h_peek) (void)hipHostFree(c->h_peek);
        c->h_peek = nullptr;
        c->peek_cap = 0;
        if (hipHostMalloc((void**)&c->h_peek, (size_t)c->pg * 4, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            c->h_peek = nullptr;
            return fail(c, PGH_E_OOM, "pinned peek buffer of %lld floats failed", (long long)c->pg);
        }
        c->peek_cap = (size_t)c->pg;
    }
    peek_job_wait(c);  // the last peek's payload copy reads h_peek
    const hipStream_t s = c->stream;  // (the last peek's D2H from d_peek has finished: queried above)
    pgh::FedavgArgs a{};
    a.diffs = (const float*)c->d_slab;
    a.map = slab_map(c);
    a.n_rows = 0;
    a.client0 = c->folded;
    a.p = c->pg;
    a.acc = c->d_acc;
    a.acc_in = c->acc_src;  // a rewound state is read where it was saved
    a.ckpt = c->d_ckpt;
    a.out = c->d_peek;
    a.divisor = fa.divisor;
    a.flags = pgh::FL_FINAL;
    a.mode = mode;
    a.variant = c->variant;
    pgh::RowTab tab{};
    const uint64_t bytes = 12ull * (uint64_t)c->pg;
    RC(timed_launch(c, s, bytes, [&] { return pgh::launch_fedavg_rows(a, tab, s); }));
    RC(record_fold(c, s));  // a checkpoint upload waits for this read of d_ckpt
    CK(c, hipEventRecord(c->peek_ev, s));
    CK(c, hipStreamWaitEvent(c->peek_stream, c->peek_ev, 0));
    const size_t total = (size_t)c->pg * 4, np = (total + D2H_PIECE - 1) / D2H_PIECE;
    while (c->peek_piece_ev.size() < np) {
        hipEvent_t e = nullptr;
        CK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->peek_piece_ev.push_back(e);
    }
    for (size_t k = 0; k < np; ++k) {
        const size_t off = k * D2H_PIECE, len = std::min(D2H_PIECE, total - off);
        CK(c, hipMemcpyAsync((uint8_t*)c->h_peek + off, (const uint8_t*)c->d_peek + off, len, hipMemcpyDeviceToHost,
                             c->peek_stream));
        CK(c, hipEventRecord(c->peek_piece_ev[k], c->peek_stream));
    }
    c->peek_pieces = np;
    CK(c, hipEventRecord(c->peek_ev, c->peek_stream));
    c->peek_gen = c->state_gen;
    return PGH_OK;
}


int pgh_fold_peek_into(pgh_ctx* c, int mode, uint8_t* out, size_t n) {
    if (c && c->grp) return pgh_group_api::fold_peek_into(c, mode, out, n);
    if (!c) return PGH_E_ARG;
    std::vector<std::pair<size_t, size_t>> spans;
    if (out) RC(state_shard_spans(c, out, n, &spans, "peek output frame"));
    {
        // a copy into another output (a cycle that ended without a close) finishes first: the
        // caller keeps only the output of its latest peek alive
        std::unique_lock<std::mutex> lk(c->pk_mu);
        c->pk_cv.wait(lk, [c, out] { return !c->pk_busy || c->pk_out == out; });
    }
    RC(pgh_fold_peek(c, mode));
    if (!out || !pgh_int::peek_valid(c)) return PGH_OK;  // skipped: nothing to copy
    // 8 threads: a piece's copy-out keeps pace with its PCIe D2H (4 were slower than the link)
    if (!c->pool_peek) c->pool_peek.reset(new CopyPool(std::min(8, std::max(1, c->copy_threads)), c->local_cpus));
    if (!c->pk_thread.joinable()) c->pk_thread = std::thread(peek_thread_main, c);
    {
        std::lock_guard<std::mutex> lk(c->pk_mu);
        c->pk_pieces.clear();
        for (auto& sp : spans) c->pk_pieces.push_back({out + sp.first, sp.second});
        c->pk_out = out;
        c->pk_gen = c->peek_gen;
        c->pk_done_gen = 0;
        c->pk_busy = true;
    }
    c->pk_cv.notify_all();
    return PGH_OK;
}

int pgh_peek_patch_state(pgh_ctx* c, uint8_t* out, size_t n, int* ok) {
    if (c && c->grp) return pgh_group_api::peek_patch_state(c, out, n, ok);
    if (!c || !ok || !out) return PGH_E_ARG;
    *ok = 0;
    if (!pgh_int::peek_valid(c)) {
        peek_job_wait(c);  // the caller may reuse `out` once this returns
        return PGH_OK;
    }
    const double t0 = now_ms();
    RC(pgh_int::peek_commit(c, out, n, out));
    c->st.close_ms_last = now_ms() - t0;
    *ok = 1;
    return PGH_OK;
}

int pgh_peek_valid(pgh_ctx* c, int* valid) {
    if (c && c->grp) return pgh_group_api::peek_valid(c, valid);
    if (!c || !valid) return PGH_E_ARG;
    *valid = pgh_int::peek_valid(c) ? 1 : 0;
    return PGH_OK;
}

int pgh_fold_busy(pgh_ctx* c, int* busy) {
    if (c && c->grp) return pgh_group_api::fold_busy(c, busy);
    if (!c || !busy) return PGH_E_ARG;
    *busy = 0;
    if (c->slot_ring.empty()) return PGH_OK;
    const hipError_t q = hipEventQuery(c->slot_ring.back().second);
    if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        *busy = 1;
    } else if (q != hipSuccess) {
        return fail(c, PGH_E_HIP, "hipEventQuery failed: %s", hipGetErrorString(q));
    }
    return PGH_OK;
}

int pgh_fold_slots_restart(pgh_ctx* c) {
    if (c && c->grp) return pgh_group_api::fold_restart(c);
    if (!c) return PGH_E_ARG;
    RC(check_slot_folds(c));
    // The next slot fold's FL_FIRST pass overwrites the fold state on c->stream, behind any fold
    // still in flight there: nothing to wait for.  Saved fold states are kept.
    c->acc_src = nullptr;
    c->folded = 0;
    c->st.n_folded = 0;
    c->slot_mode = -1;
    ++c->state_gen;
    c->weights.clear();
    c->weights_on_device = false;
    return PGH_OK;
}

