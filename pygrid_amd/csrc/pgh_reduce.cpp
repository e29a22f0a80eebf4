// libpygrid_hip: RESIDENT folds (every ingested client in one launch, repeatable), the resident
// checkpoint kept in HBM across cycles, secure aggregation (Z_2^64 share sum + fixed-point decode) and
// STREAM folds (a ring of slots folded in client order while ingest continues).  Reference:
// cycle_manager.py:252-296 (fedavg), test_basic_syft_operations.py:417-424 (secagg).
// (struct pgh_ctx and the shared helpers: pgh_ctx.h)
#include "pgh_ctx.h"

using namespace pgh_detail;

// (the public entry points take their C linkage from include/pgh_api.h)

// ---- RESIDENT reductions -------------------------------------------------------------------------

int pgh_fedavg_device(pgh_ctx* c, int mode, const float* d_ckpt, float* d_out, void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    RC(check_dtype(c, PGH_F32));
    if (!valid_mode(mode)) return fail(c, PGH_E_ARG, "unknown averaging mode %d", mode);
    if (!d_ckpt || !d_out) return fail(c, PGH_E_ARG, "d_ckpt / d_out is NULL");
    if (((uintptr_t)d_ckpt | (uintptr_t)d_out) & 15) return fail(c, PGH_E_ARG, "device buffers must be 16-byte aligned");
    DeviceGuard g(c->device);
    int64_t n = 0;
    RC(resident_count(c, &n));
    FinalArgs fa;
    fa.ckpt = d_ckpt;
    fa.out = d_out;
    RC(fedavg_divisor(c, mode, n, &fa.divisor));
    hipStream_t s = (hipStream_t)stream;
    return fold_run(c, mode, 0, n, true, fa, s);
}

int pgh_fedavg_device_range(pgh_ctx* c, int mode, int64_t off, int64_t len, const float* d_ckpt, float* d_out,
                            void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    RC(check_dtype(c, PGH_F32));
    if (!valid_mode(mode)) return fail(c, PGH_E_ARG, "unknown averaging mode %d", mode);
    if (!d_ckpt || !d_out || (((uintptr_t)d_ckpt | (uintptr_t)d_out) & 15))
        return fail(c, PGH_E_ARG, "d_ckpt / d_out must be 16-byte aligned device pointers");
    DeviceGuard g(c->device);
    int64_t n = 0;
    RC(resident_count(c, &n));
    FinalArgs fa;
    fa.ckpt = d_ckpt;
    fa.out = d_out;
    fa.off = off;
    fa.len = len;
    RC(fedavg_divisor(c, mode, n, &fa.divisor));
    return fold_run(c, mode, 0, n, true, fa, (hipStream_t)stream);
}

int pgh_fedavg(pgh_ctx* c, int mode, const float* ckpt, float* out) {
    if (c && c->grp) return pgh_group_api::fedavg(c, mode, ckpt, out);
    RC(check_dtype(c, PGH_F32));
    if (!ckpt || !out) return fail(c, PGH_E_ARG, "ckpt / out is NULL");
    DeviceGuard g(c->device);
    const double t0 = now_ms();
    const size_t bytes = sizeof(float) * (size_t)c->pg;
    RC(order_before_overwrite(c));
    c->ckpt_valid = false;
    clear_final_marks(c);
    RC(stage_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), (const uint8_t*)ckpt, bytes, is_pinned(ckpt)));
    c->ckpt_valid = true;
    RC(pgh_fedavg_device(c, mode, c->d_ckpt, c->d_out, c->stream));
    if (is_pinned(out)) {
        CK(c, hipMemcpyAsync(out, c->d_out, bytes, hipMemcpyDeviceToHost, c->stream));
        CK(c, hipStreamSynchronize(c->stream));
    } else {
        RC(stage_d2h_pieces(c, (const uint8_t*)c->d_out, {OutPiece{(uint8_t*)out, bytes}}, c->stream));
    }
    c->st.close_ms_last = now_ms() - t0;
    return collect_timings(c);
}

// ---- resident checkpoint: the new checkpoint stays in HBM as the next cycle's input ------------

int pgh_ckpt_upload(pgh_ctx* c, const float* ckpt, size_t nbytes) {
    if (c && c->grp) return pgh_group_api::ckpt_upload(c, ckpt, nbytes);
    RC(check_dtype(c, PGH_F32));
    if (!ckpt) return fail(c, PGH_E_ARG, "ckpt is NULL");
    const size_t whole = 4 * (size_t)c->P, shard = 4 * (size_t)c->pg;
    if (nbytes != whole && nbytes != shard)
        return fail(c, PGH_E_ARG, "checkpoint: got %zu bytes, layout needs %zu (model) or %zu (shard)", nbytes, whole,
                    shard);
    DeviceGuard g(c->device);
    RC(order_before_overwrite(c));
    const uint8_t* src = (const uint8_t*)ckpt + (nbytes == whole ? 4 * (size_t)c->lo : 0);
    c->ckpt_valid = false;
    clear_final_marks(c);
    RC(stage_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), src, shard, is_pinned(ckpt)));
    c->ckpt_valid = true;
    return PGH_OK;
}

int pgh_ckpt_upload_state(pgh_ctx* c, const uint8_t* pb, size_t n) {
    if (c && c->grp) return pgh_group_api::ckpt_upload_state(c, pb, n);
    RC(check_dtype(c, PGH_F32));
    if (!pb && n) return fail(c, PGH_E_ARG, "pb is NULL");
    std::vector<std::pair<size_t, size_t>> spans;
    RC(state_shard_spans(c, pb, n, &spans, "checkpoint"));
    std::vector<Piece> pieces;
    for (auto& sp : spans) pieces.push_back(Piece{pb + sp.first, sp.second});
    DeviceGuard g(c->device);
    RC(order_before_overwrite(c));
    c->ckpt_valid = false;
    clear_final_marks(c);
    RC(stage_pieces_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), pieces));
    c->ckpt_valid = true;
    return PGH_OK;
}

int pgh_fedavg_resident(pgh_ctx* c, int mode) {
    if (c && c->grp) return pgh_group_api::fedavg_resident(c, mode);
    RC(check_dtype(c, PGH_F32));
    RC(check_ckpt(c, "pgh_fedavg_resident"));
    if (!valid_mode(mode)) return fail(c, PGH_E_ARG, "unknown averaging mode %d", mode);
    DeviceGuard g(c->device);
    const double t0 = now_ms();
    clear_final_marks(c);
    const int K = final_ranges(c);
    if (K == 1) {
        RC(pgh_fedavg_device(c, mode, c->d_ckpt, c->d_out, c->stream));
    } else {  // the same fold as K range launches, each followed by its mark (pipelined close)
        int64_t n = 0;
        RC(resident_count(c, &n));
        FinalArgs fa;
        fa.ckpt = c->d_ckpt;
        fa.out = c->d_out;
        RC(fedavg_divisor(c, mode, n, &fa.divisor));
        RC(fork_aux(c, c->stream));
        for (int k = 0; k < K; ++k) {
            fa.off = range_edge(c, k, K);
            fa.len = range_edge(c, k + 1, K) - fa.off;
            const hipStream_t rs = range_stream(c, c->stream, k);
            RC(fold_run(c, mode, 0, n, true, fa, rs));
            RC(add_final_mark(c, rs, fa.off + fa.len));
        }
        RC(join_aux(c, c->stream));
    }
    std::swap(c->d_ckpt, c->d_out);  // the new checkpoint is the next cycle's input
    c->st.close_ms_last = now_ms() - t0;
    return PGH_OK;
}

int pgh_ckpt_download(pgh_ctx* c, float* out) {
    if (c && c->grp) return pgh_group_api::ckpt_download(c, out);
    RC(check_dtype(c, PGH_F32));
    if (!out) return fail(c, PGH_E_ARG, "out is NULL");
    RC(check_ckpt(c, "pgh_ckpt_download"));
    DeviceGuard g(c->device);
    const size_t bytes = 4 * (size_t)c->pg;
    RC(order_after_ingest(c, c->stream));
    if (is_pinned(out)) {
        CK(c, hipMemcpyAsync(out, c->d_ckpt, bytes, hipMemcpyDeviceToHost, c->stream));
        CK(c, hipStreamSynchronize(c->stream));
    } else {
        RC(stage_d2h_pieces(c, (const uint8_t*)c->d_ckpt, {OutPiece{(uint8_t*)out, bytes}}, c->stream, nullptr, true));
    }
    return collect_timings(c);
}

int pgh_ckpt_patch_state(pgh_ctx* c, const uint8_t* tmpl, size_t n, uint8_t* out) {
    if (c && c->grp) return pgh_group_api::ckpt_patch_state(c, tmpl, n, out);
    RC(check_dtype(c, PGH_F32));
    if (!tmpl || !out) return fail(c, PGH_E_ARG, "tmpl / out is NULL");
    RC(check_ckpt(c, "pgh_ckpt_patch_state"));
    std::vector<std::pair<size_t, size_t>> spans;
    RC(state_shard_spans(c, tmpl, n, &spans, "checkpoint template"));
    DeviceGuard g(c->device);
    std::vector<CopyPool::Seg> gaps;
    bool ordered = true;
    if (out != tmpl) {  // template bytes outside this shard's payload slices (framing, other shards)
        size_t pos = 0;
        for (auto& sp : spans) {
            ordered = ordered && sp.first >= pos;
            if (sp.first > pos) gaps.push_back({out + pos, tmpl + pos, sp.first - pos});
            pos = sp.first + sp.second;
        }
        if (n > pos) gaps.push_back({out + pos, tmpl + pos, n - pos});
    }
    std::vector<OutPiece> pieces;
    for (auto& sp : spans) pieces.push_back(OutPiece{out + sp.first, sp.second});
    RC(order_after_ingest(c, c->stream));
    if (!ordered) {  // overlapping spans (never from the walker): whole template first, then payloads
        c->pool_copy->run({CopyPool::Seg{out, tmpl, n}});
        gaps.clear();
    }
    // the framing copy and the pre-fault of the output run while the first slot's DMA flies (in
    // place, out == tmpl, is how a freshly framed checkpoint is filled: its pages are fresh too)
    RC(stage_d2h_pieces(c, (const uint8_t*)c->d_ckpt, pieces, c->stream, [&] {
        prefault_parallel(out, n, *c->pool_copy);
        if (!gaps.empty()) c->pool_copy->run(gaps);
    }, true));
    return collect_timings(c);
}

int pgh_secagg_device(pgh_ctx* c, int base, int prec, int64_t* d_sum, float* d_dec, void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    RC(check_dtype(c, PGH_I64));
    DeviceGuard g(c->device);
    int64_t n = 0;
    RC(resident_count(c, &n));
    FinalArgs fa;
    fa.sum = d_sum;
    fa.dec = d_dec;
    RC(fixed_point_divisor(c, base, prec, &fa.divisor));
    return fold_run(c, KIND_SECAGG, 0, n, true, fa, (hipStream_t)stream);
}

int pgh_secagg_device_range(pgh_ctx* c, int base, int prec, int64_t off, int64_t len, int64_t* d_sum, float* d_dec,
                            void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    RC(check_dtype(c, PGH_I64));
    DeviceGuard g(c->device);
    int64_t n = 0;
    RC(resident_count(c, &n));
    FinalArgs fa;
    fa.sum = d_sum;
    fa.dec = d_dec;
    fa.off = off;
    fa.len = len;
    RC(fixed_point_divisor(c, base, prec, &fa.divisor));
    return fold_run(c, KIND_SECAGG, 0, n, true, fa, (hipStream_t)stream);
}

int pgh_secagg_decode_device(pgh_ctx* c, int base, int prec, const int64_t* d_sum, int64_t n, float* d_dec,
                             void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    if (!c) return fail(nullptr, PGH_E_ARG, "null context");
    if (n < 0 || (n > 0 && (!d_sum || !d_dec))) return fail(c, PGH_E_ARG, "bad decode arguments (n=%lld)", (long long)n);
    DeviceGuard g(c->device);
    float div = 1.f;
    RC(fixed_point_divisor(c, base, prec, &div));
    const hipStream_t s = (hipStream_t)stream;
    // not in pgh_stats' kernel timings: those stay the share-sum / fold kernels' (12 B per param here)
    const hipError_t e = pgh::launch_secagg_decode(d_sum, d_dec, n, div, s);
    if (e != hipSuccess) return fail(c, PGH_E_HIP, "decode launch failed: %s", hipGetErrorString(e));
    return PGH_OK;
}

int pgh_secagg(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out) {
    if (c && c->grp) return pgh_group_api::secagg(c, base, prec, sum_out, dec_out);
    RC(check_dtype(c, PGH_I64));
    DeviceGuard g(c->device);
    const double t0 = now_ms();
    RC(pgh_secagg_device(c, base, prec, sum_out ? c->d_sum : nullptr, dec_out ? c->d_dec : nullptr, c->stream));
    if (sum_out) CK(c, hipMemcpyAsync(sum_out, c->d_sum, 8ull * c->pg, hipMemcpyDeviceToHost, c->stream));
    if (dec_out) CK(c, hipMemcpyAsync(dec_out, c->d_dec, 4ull * c->pg, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->st.close_ms_last = now_ms() - t0;
    return collect_timings(c);
}

// ---- STREAM reductions ---------------------------------------------------------------------------

int pgh_stream_begin(pgh_ctx* c, int kind, int fold_batch) {
    if (c && c->grp) return pgh_group_api::stream_begin(c, kind, fold_batch);
    RC(check_ready(c));
    if (kind == PGH_STREAM_SECAGG) {
        if (c->dtype != PGH_I64) return fail(c, PGH_E_STATE, "secagg stream needs an int64 slab");
    } else if (!valid_mode(kind) || c->dtype != PGH_F32) {
        return fail(c, PGH_E_ARG, "stream kind %d does not match the slab", kind);
    }
    DeviceGuard g(c->device);
    RC(pgh_reset(c));
    c->streaming = true;
    c->kind = kind == PGH_STREAM_SECAGG ? KIND_SECAGG : kind;
    c->fold_batch = fold_batch <= 0 ? std::max(1, c->slots / 2) : std::min(fold_batch, c->slots);
    return PGH_OK;
}

int pgh_stream_flush(pgh_ctx* c) {
    if (c && c->grp) return pgh_group_api::stream_flush(c);
    RC(check_ready(c));
    if (!c->streaming) return fail(c, PGH_E_STATE, "not streaming");
    DeviceGuard g(c->device);
    return maybe_fold(c, true);
}

namespace {
int stream_finish(pgh_ctx* c, FinalArgs fa, hipStream_t cs, bool fedavg, int mode_or_base) {
    if (!c->streaming) return fail(c, PGH_E_STATE, "not streaming (call pgh_stream_begin first)");
    const int64_t run = ready_run(c, c->folded);
    RC(check_no_gaps(c, c->folded, run));
    const int64_t n = c->folded + run;
    if (n == 0) return fail(c, PGH_E_STATE, "no diffs ingested");
    if (fedavg) RC(fedavg_divisor(c, mode_or_base, n, &fa.divisor));
    RC(join_in(c, cs));
    RC(fold_run(c, c->kind, c->folded, run, true, fa, c->stream));
    RC(join_out(c, cs));
    for (int64_t k = 0; k < run; ++k) c->slot_client[(size_t)((c->folded + k) % c->slots)] = -1;
    c->folded = n;
    c->st.n_folded = n;
    c->streaming = false;
    return PGH_OK;
}
}  // namespace

int pgh_stream_finish_device(pgh_ctx* c, const float* d_ckpt, float* d_out, void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    RC(check_dtype(c, PGH_F32));
    if (!d_ckpt || !d_out || (((uintptr_t)d_ckpt | (uintptr_t)d_out) & 15))
        return fail(c, PGH_E_ARG, "d_ckpt / d_out must be 16-byte aligned device pointers");
    DeviceGuard g(c->device);
    FinalArgs fa;
    fa.ckpt = d_ckpt;
    fa.out = d_out;
    return stream_finish(c, fa, (hipStream_t)stream, true, c->kind);
}

int pgh_stream_finish_resident(pgh_ctx* c) {
    if (c && c->grp) return pgh_group_api::stream_finish_resident(c);
    RC(check_dtype(c, PGH_F32));
    RC(check_ckpt(c, "pgh_stream_finish_resident"));
    DeviceGuard g(c->device);
    clear_final_marks(c);
    const double t0 = now_ms();
    RC(pgh_stream_finish_device(c, c->d_ckpt, c->d_out, c->stream));
    std::swap(c->d_ckpt, c->d_out);  // the new checkpoint is the next cycle's input
    c->st.close_ms_last = now_ms() - t0;
    return PGH_OK;
}

int pgh_stream_finish(pgh_ctx* c, const float* ckpt, float* out) {
    if (c && c->grp) return pgh_group_api::stream_finish(c, ckpt, out);
    RC(check_dtype(c, PGH_F32));
    if (!ckpt || !out) return fail(c, PGH_E_ARG, "ckpt / out is NULL");
    DeviceGuard g(c->device);
    const double t0 = now_ms();
    const size_t bytes = sizeof(float) * (size_t)c->pg;
    // staged like pgh_fedavg's checkpoint: on the copy stream after every fold that may still read
    // d_ckpt, so fold_run's order_after_ingest orders the final fold after it (a pageable
    // pgh_ckpt_upload's last ring DMA can no longer land after this copy)
    RC(order_before_overwrite(c));
    c->ckpt_valid = false;
    clear_final_marks(c);
    RC(stage_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), (const uint8_t*)ckpt, bytes, is_pinned(ckpt)));
    c->ckpt_valid = true;
    RC(pgh_stream_finish_device(c, c->d_ckpt, c->d_out, c->stream));
    CK(c, hipMemcpyAsync(out, c->d_out, bytes, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->st.close_ms_last = now_ms() - t0;
    return collect_timings(c);
}

int pgh_stream_finish_secagg_device(pgh_ctx* c, int base, int prec, int64_t* d_sum, float* d_dec, void* stream) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    RC(check_dtype(c, PGH_I64));
    DeviceGuard g(c->device);
    FinalArgs fa;
    fa.sum = d_sum;
    fa.dec = d_dec;
    RC(fixed_point_divisor(c, base, prec, &fa.divisor));
    return stream_finish(c, fa, (hipStream_t)stream, false, base);
}

int pgh_stream_finish_secagg(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out) {
    if (c && c->grp) return pgh_group_api::stream_finish_secagg(c, base, prec, sum_out, dec_out);
    RC(check_dtype(c, PGH_I64));
    DeviceGuard g(c->device);
    const double t0 = now_ms();
    RC(pgh_stream_finish_secagg_device(c, base, prec, sum_out ? c->d_sum : nullptr, dec_out ? c->d_dec : nullptr,
                                       c->stream));
    if (sum_out) CK(c, hipMemcpyAsync(sum_out, c->d_sum, 8ull * c->pg, hipMemcpyDeviceToHost, c->stream));
    if (dec_out) CK(c, hipMemcpyAsync(dec_out, c->d_dec, 4ull * c->pg, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->st.close_ms_last = now_ms() - t0;
    return collect_timings(c);
}

