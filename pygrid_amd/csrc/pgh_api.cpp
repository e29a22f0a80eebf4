// libpygrid_hip: C-ABI context around the gfx950 aggregation kernels.
//
// One pgh_ctx = one GPU = one parameter shard.  It owns
//   * the HBM slab: R slots x rows_per_client rows (fp32 diffs, or n_parties int64 share rows
//     per client), column-blocked: the shard is cut into blocks of bw columns (256 KiB of one
//     row by default) and each block stores all rows one after another (SlabMap in
//     pgh_kernels.h), so a kernel lane walking down the rows of its column stays in one block;
//   * the [P_shard] device vectors (checkpoint, output, running fold state, weights);
//   * a 2-slot pinned host ring through which pageable host bytes reach the slab
//     (multi-threaded host memcpy into a pinned slot overlapping the previous slot's DMA on a
//     dedicated copy stream); page-locked caller buffers are DMA'd directly;
//   * HIP event pairs around every reduction launch (pgh_stats reports kernel time).
//
// Two ways to use the slab:
//   RESIDENT  client k lives in slot k until the context is reset; pgh_fedavg / pgh_secagg fold
//             all clients [0, n) in one launch (repeatable: the diffs stay resident).
//   STREAM    (pgh_stream_begin .. pgh_stream_finish) client k goes to slot k % R; every run of
//             consecutive clients starting at the fold front is folded into the running state
//             (in client order, so fp32 results are bit-identical to RESIDENT) and its slots
//             freed.  Lets N x P exceed HBM and overlaps H2D ingest with reduction (SURVEY 8(d)
//             configs 3-5) and folds diffs as they are reported.
//
// Reference mapping: ingest = the N x unserialize_model_params loop of
// cycle_manager.py:247-250; fedavg = :252-296; secagg = PySyft share add + .get() + float_prec
// (test_basic_syft_operations.py:417-424).  Errors are negative status codes plus a message (the
// Python shim raises a PyGridError subclass, as tasks/cycle.py:33-37 expects).
//
// This file: lifecycle, page-locked host blocks, observability, the helpers every entry point shares
// (declared in pgh_ctx.h) and the group driver's internals.  pgh_ingest.cpp, pgh_reduce.cpp and
// pgh_slots.cpp hold the rest of the entry points.
#include <emmintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <fstream>

#include "pgh_ctx.h"

namespace pgh_detail {

void copy_stream(uint8_t* dst, const uint8_t* src, size_t n) {
    if (n < (256u << 10)) { std::memcpy(dst, src, n); return; }
    const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
    std::memcpy(dst, src, head);
    dst += head; src += head; n -= head;
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

void bind_thread(const std::vector<int>& cpus) {
    if (cpus.empty()) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
}

std::vector<int> gpu_local_cpus(int device) {
    std::vector<int> out;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) { (void)hipGetLastError(); return out; }
    std::string id(bus);
    for (auto& ch : id) ch = (char)std::tolower((unsigned char)ch);
    std::ifstream f("/sys/bus/pci/devices/" + id + "/local_cpulist");
    std::string list;
    if (!f || !std::getline(f, list)) return out;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return out;
    size_t pos = 0;
    while (pos < list.size()) {
        size_t end = list.find(',', pos);
        if (end == std::string::npos) end = list.size();
        const std::string r = list.substr(pos, end - pos);
        const size_t dash = r.find('-');
        const int a = std::atoi(r.c_str()), b = dash == std::string::npos ? a : std::atoi(r.c_str() + dash + 1);
        for (int cpu = a; cpu <= b && cpu < CPU_SETSIZE; ++cpu)
            if (cpu >= 0 && CPU_ISSET(cpu, &allowed)) out.push_back(cpu);
        pos = end + 1;
    }
    return out;
}

thread_local std::string g_create_err;

int vfail(pgh_ctx* c, int code, const char* fmt, va_list ap) {
    char buf[1024];
    vsnprintf(buf, sizeof buf, fmt, ap);
    if (c) c->err = buf; else g_create_err = buf;
    return code;
}

int fail(pgh_ctx* c, int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const int r = vfail(c, code, fmt, ap);
    va_end(ap);
    return r;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void free_slab(pgh_ctx* c) {
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    if (c->dec) (void)hipStreamSynchronize(c->dec);  // a varint decode writes slab rows
    for (auto& fe : c->fold_evs) (void)hipEventSynchronize(fe.second);  // folds on caller streams
    (void)hipFree(c->d_slab); c->d_slab = nullptr; c->slab_bytes = 0;
    (void)hipFree(c->d_ckpt); c->d_ckpt = nullptr;
    (void)hipFree(c->d_out); c->d_out = nullptr;
    c->ckpt_valid = false;
    for (auto& m : c->final_marks) c->rmark_pool.push_back(m.ev);
    c->final_marks.clear();
    c->pre_d2h_valid = false;
    (void)hipFree(c->d_acc); c->d_acc = nullptr;
    (void)hipFree(c->d_uacc); c->d_uacc = nullptr;
    (void)hipFree(c->d_sum); c->d_sum = nullptr;
    (void)hipFree(c->d_dec); c->d_dec = nullptr;
    (void)hipFree(c->d_w); c->d_w = nullptr; c->w_cap = 0;
    c->slots = 0;
    c->slot_mode = -1;
    c->slot_client.clear();
    for (auto& m : c->marks) c->mark_pool.push_back(m.ev);
    c->marks.clear();
    c->streaming = false;
    c->folded = 0;
    for (auto& fe : c->fold_evs) c->fold_ev_pool.push_back(fe.second);
    c->fold_evs.clear();
    release_slot_fold_events(c);
    c->slot_read_seq.clear();
    c->weights_on_device = false;
}

int check_ready(pgh_ctx* c) {
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (!c->d_slab) return fail(c, PGH_E_STATE, "pgh_reserve has not been called");
    return PGH_OK;
}

int check_dtype(pgh_ctx* c, int dtype) {
    RC(check_ready(c));
    if (c->dtype != dtype) return fail(c, PGH_E_STATE, "slab holds dtype %d, call needs %d", c->dtype, dtype);
    return PGH_OK;
}

int check_ckpt(pgh_ctx* c, const char* what) {
    if (!c->ckpt_valid)
        return fail(c, PGH_E_STATE, "%s: no checkpoint in HBM (pgh_ckpt_upload* since the last pgh_reserve / layout "
                    "change)", what);
    return PGH_OK;
}

// Columns per block for a shard of pg elements of es bytes: one block when the whole row fits
// in block_bytes (or blocking is off), else the widest power of two <= block_bytes whose
// padding of the last block stays within 1/16 of the row.
void slab_geometry(int64_t pg, size_t es, size_t block_bytes, int64_t* bw, int64_t* nb, int* bshift) {
    const int64_t whole = (pg + 63) & ~(int64_t)63;
    int64_t maxc = 64;
    while (maxc * 2 * (int64_t)es <= (int64_t)block_bytes) maxc *= 2;
    if (block_bytes == 0 || whole <= maxc) { *bw = whole; *nb = 1; *bshift = 62; return; }
    int64_t b = maxc;
    while (b > 64 && ((pg + b - 1) / b) * b - pg > pg / 16) b /= 2;
    *bw = b;
    *nb = (pg + b - 1) / b;
    int sh = 0;
    while ((int64_t(1) << sh) < b) ++sh;
    *bshift = sh;
}

// Elements [i0, i0 + n) of one row from contiguous host memory: the partial first block, the
// whole blocks as ONE 2-D copy (block rows bstride apart), the partial last block.
int h2d_range(pgh_ctx* c, const Dest& d, int64_t i0, const uint8_t* src, int64_t n, hipStream_t s,
              size_t src_room) {
    const size_t es = d.es;
    if (n <= 0) return PGH_OK;
    ++c->copy_seq;
    if (d.map.bshift == 62) {
        CK(c, hipMemcpyAsync(d.base + (size_t)i0 * es, src, (size_t)n * es, hipMemcpyHostToDevice, s));
        return PGH_OK;
    }
    const int64_t bw = d.map.ld, i1 = i0 + n;
    int64_t i = i0;
    if (i & (bw - 1)) {  // head
        const int64_t e = std::min(i1, (i | (bw - 1)) + 1);
        CK(c, hipMemcpyAsync(d.base + (size_t)d.map.at(i) * es, src, (size_t)(e - i) * es, hipMemcpyHostToDevice, s));
        src += (size_t)(e - i) * es;
        i = e;
    }
    int64_t full = (i1 - i) / bw;
    const int64_t rest = (i1 - i) - full * bw;
    const bool pad = rest > 0 && d.len > 0 && i1 == d.len && src_room >= (size_t)(bw - rest) * es;
    if (pad) ++full;  // the row's partial last block as a whole one: one copy less per row
    if (full > 0) {
        CK(c, hipMemcpy2DAsync(d.base + (size_t)d.map.at(i) * es, (size_t)d.map.bstride * es, src, (size_t)bw * es,
                               (size_t)bw * es, (size_t)full, hipMemcpyHostToDevice, s));
        src += (size_t)(full * bw) * es;
        i = std::min(i1, i + full * bw);
    }
    if (i < i1)  // tail
        CK(c, hipMemcpyAsync(d.base + (size_t)d.map.at(i) * es, src, (size_t)(i1 - i) * es, hipMemcpyHostToDevice, s));
    return PGH_OK;
}

// Timing events (timed_launch) only measure: no system-scope fence when they complete.  With the
// default flags each one made the kernel after it start 15-22 us after the one before, against 5-7
// without (tools/exp_close_pipeline.hip, profiles/r05e/): 12 range launches of a report-time close
// lost ~0.15 ms to them.  Every host read of a result still goes through a copy with its own sync.
hipEvent_t take_event(pgh_ctx* c) {
    if (!c->pool.empty()) { hipEvent_t e = c->pool.back(); c->pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

int collect_timings(pgh_ctx* c) {
    // busy time: union of the launches' intervals, placed on one clock relative to the first start
    std::vector<std::pair<double, double>> iv;
    iv.reserve(c->pending.size());
    for (auto& t : c->pending) {
        CK(c, hipEventSynchronize(t.b));
        float ms = 0.f, t0 = 0.f;
        CK(c, hipEventElapsedTime(&ms, t.a, t.b));
        CK(c, hipEventElapsedTime(&t0, c->pending.front().a, t.a));
        iv.push_back({(double)t0, (double)t0 + ms});
        c->st.kernel_ms_last = ms;
        c->st.kernel_ms_total += ms;
        c->st.kernel_launches += 1;
        c->st.kernel_bytes_last = t.bytes;
        c->st.kernel_bytes_total += t.bytes;
        c->pool.push_back(t.a);
        c->pool.push_back(t.b);
    }
    c->pending.clear();
    std::sort(iv.begin(), iv.end());
    double busy = 0, lo = 0, hi = 0;
    bool open = false;
    for (auto& x : iv) {
        if (open && x.first <= hi) { hi = std::max(hi, x.second); continue; }
        if (open) busy += hi - lo;
        lo = x.first; hi = x.second; open = true;
    }
    if (open) busy += hi - lo;
    c->st.kernel_busy_ms_total += busy;
    return PGH_OK;
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    return attr.type == hipMemoryTypeHost;
}

// Ranged report ingest (pgh_set_ingest_ranges) of concatenated fp32 host pieces holding the whole
// shard row: one pinned slot, filled and DMA'd chunk by chunk (INGEST_CHUNK params each, the host
// copy of chunk k + 1 beside the DMA of chunk k), rng_ev[k] behind chunk k's DMA.
int stage_pieces_h2d_ranged(pgh_ctx* c, const Dest& dst, const std::vector<Piece>& pieces, size_t total) {
    const double t0 = now_ms();
    const int K = (int)((c->pg + INGEST_CHUNK - 1) / INGEST_CHUNK);
    while ((int)c->rng_ev.size() < K) {
        hipEvent_t e = nullptr;
        CK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->rng_ev.push_back(e);
    }
    int slot = 0;
    RC(take_pin_slot(c, &slot));
    size_t pi = 0, poff = 0;
    for (int k = 0; k < K; ++k) {
        const size_t a = (size_t)k * INGEST_CHUNK * 4, b = std::min(total, (size_t)(k + 1) * INGEST_CHUNK * 4);
        std::vector<CopyPool::Seg> segs;
        for (size_t at = a; at < b;) {
            const size_t m = std::min(pieces[pi].n - poff, b - at);
            segs.push_back({c->h_pin[slot] + at, pieces[pi].src + poff, m});
            at += m;
            poff += m;
            if (poff == pieces[pi].n) { ++pi; poff = 0; }
        }
        c->pool_copy->run(segs);
        RC(h2d_range(c, dst, (int64_t)(a / 4), c->h_pin[slot] + a, (int64_t)((b - a) / 4), c->copy,
                     b == total ? c->pin_slot - b : 0));
        CK(c, hipEventRecord(c->rng_ev[(size_t)k], c->copy));
    }
    CK(c, hipEventRecord(c->pin_ev[slot], c->copy));
    c->pin_used[slot] = true;
    c->rng_seq = c->copy_seq;
    c->rng_n = K;
    c->st.h2d_ms_total += now_ms() - t0;
    c->st.h2d_bytes_total += total;
    c->st.h2d_staged_bytes_total += total;
    return PGH_OK;
}

// Whether the FINAL pass of a slot fold may wait per param range on the latest ranged ingest
// instead of on every copy issued (order_after_ingest): nothing else went to the copy stream since.
bool ranged_ingest_valid(const pgh_ctx* c) {
    return c->ingest_ranges && c->rng_seq == c->copy_seq && c->rng_n == (int)((c->pg + INGEST_CHUNK - 1) / INGEST_CHUNK);
}

// Concatenated host pieces -> HBM at `dst`, through the pinned ring: each slot is filled by
// (multi-threaded) host copies of as many pieces as fit, then DMA'd while the next slot fills.
int stage_pieces_h2d(pgh_ctx* c, const Dest& dst, const std::vector<Piece>& pieces) {
    const double t0 = now_ms();
    size_t total = 0, done = 0, pi = 0, poff = 0;
    for (auto& p : pieces) total += p.n;
    while (done < total) {
        int slot = 0;
        RC(take_pin_slot(c, &slot));
        size_t fill = 0;
        std::vector<CopyPool::Seg> segs;
        while (fill < c->pin_slot && pi < pieces.size()) {
            const size_t m = std::min(pieces[pi].n - poff, c->pin_slot - fill);
            segs.push_back({c->h_pin[slot] + fill, pieces[pi].src + poff, m});
            fill += m;
            poff += m;
            if (poff == pieces[pi].n) { ++pi; poff = 0; }
        }
        c->pool_copy->run(segs);
        // slot fills are whole multiples of 4 KiB but the last, so `done` stays element-aligned
        RC(h2d_range(c, dst, (int64_t)(done / dst.es), c->h_pin[slot], (int64_t)(fill / dst.es), c->copy,
                     c->pin_slot - fill));
        CK(c, hipEventRecord(c->pin_ev[slot], c->copy));
        c->pin_used[slot] = true;
        done += fill;
    }
    c->st.h2d_ms_total += now_ms() - t0;
    c->st.h2d_bytes_total += total;
    c->st.h2d_staged_bytes_total += total;
    return PGH_OK;
}

// host bytes -> HBM on the copy stream.  Page-locked sources are DMA'd directly (the call
// then waits for the copy: the caller's buffer is only borrowed); pageable sources go through
// the pinned ring, so the host memcpy of one slot overlaps the DMA of the other.
int stage_h2d(pgh_ctx* c, const Dest& dst, const uint8_t* src, size_t n, bool pinned_src) {
    if (!pinned_src) return stage_pieces_h2d(c, dst, {Piece{src, n}});
    const double t0 = now_ms();
    RC(h2d_range(c, dst, 0, src, (int64_t)(n / dst.es), c->copy));
    CK(c, hipStreamSynchronize(c->copy));
    c->st.h2d_ms_total += now_ms() - t0;
    c->st.h2d_bytes_total += n;
    return PGH_OK;
}

// Copy bytes [off, off + len) of the concatenation of `pieces` from `src`.
void scatter_out(const uint8_t* src, size_t off, size_t len, const std::vector<OutPiece>& pieces, CopyPool& pool) {
    std::vector<CopyPool::Seg> segs;
    size_t base = 0;
    for (auto& p : pieces) {
        const size_t a = std::max(off, base), b = std::min(off + len, base + p.n);
        if (a < b) segs.push_back({p.dst + (a - base), src + (a - off), b - a});
        base += p.n;
        if (base >= off + len) break;
    }
    pool.run(segs);
}

// Fault in the pages of a small, freshly allocated host destination with one madvise call
// (MADV_POPULATE_WRITE, Linux 5.14+) instead of one page fault per 4 KiB during the copy-out; big
// destinations are left to the copy pool, whose threads fault their own pages in parallel.  Best
// effort: an older kernel or a non-anonymous mapping just returns an error, which is ignored.
void prefault_small(uint8_t* p, size_t n) {
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
    if (!p || n == 0 || n >= (4u << 20)) return;
    static const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = (uintptr_t)p & ~(page - 1), b = ((uintptr_t)p + n + page - 1) & ~(page - 1);
    (void)madvise((void*)a, b - a, MADV_POPULATE_WRITE);
}

// MADV_POPULATE_WRITE over [p, p + n) whatever its size (pgh_host_prefault's per-thread piece).
void prefault_small_any(uint8_t* p, size_t n) {
    static const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = (uintptr_t)p & ~(page - 1), b = ((uintptr_t)p + n + page - 1) & ~(page - 1);
    (void)madvise((void*)a, b - a, MADV_POPULATE_WRITE);
}

// The same for a big fresh destination, split over the copy pool's threads: run while the fold
// and the first D2H are still in flight, so the copy-out afterwards writes to resident pages
// instead of taking a page fault per 4 KiB.
// Every page of [a, b) is already in memory (an output framed and faulted in beforehand,
// pgh_host_prefault): one mincore call, far cheaper than MADV_POPULATE_WRITE walking the same
// present pages again (≈1.6 ms for 47 MB, tools/patch_probe.py, profiles/r03l/).
bool all_resident(uintptr_t a, uintptr_t b, uintptr_t page) {
    std::vector<unsigned char> v((size_t)((b - a) / page));
    if (v.empty() || mincore((void*)a, b - a, v.data()) != 0) return false;
    for (unsigned char x : v)
        if (!(x & 1)) return false;
    return true;
}

void prefault_parallel(uint8_t* p, size_t n, CopyPool& pool) {
    if (!p || n == 0) return;
    if (n < (4u << 20)) { prefault_small(p, n); return; }
    static const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = (uintptr_t)p & ~(page - 1), b = ((uintptr_t)p + n + page - 1) & ~(page - 1);
    if (all_resident(a, b, page)) return;
    // (transparent huge pages for this range measured neutral, profiles/r02ad/: 4 KiB pages)
    const int k = pool.threads();
    const uintptr_t per = ((b - a) / k + page - 1) & ~(page - 1);
    pool.run_items(k, true, [&](int i) {
        const uintptr_t lo = a + per * (uintptr_t)i, hi = std::min(b, lo + per);
        if (lo < hi) (void)madvise((void*)lo, hi - lo, MADV_POPULATE_WRITE);
    });
}

// ---- pipelined close: range marks of the last resident fold ---------------------------------------
void clear_final_marks(pgh_ctx* c) {
    for (auto& m : c->final_marks) c->rmark_pool.push_back(m.ev);
    c->final_marks.clear();
    c->pre_d2h_valid = false;
}

int add_final_mark(pgh_ctx* c, hipStream_t s, int64_t end) {
    hipEvent_t e = nullptr;
    if (!c->rmark_pool.empty()) { e = c->rmark_pool.back(); c->rmark_pool.pop_back(); }
    else CK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(c, hipEventRecord(e, s));
    c->final_marks.push_back({end, e});
    return PGH_OK;
}

// The ranges of a split FINAL pass alternate over `s` and the aux stream, so range k + 1 starts
// while range k drains its last workgroups instead of after (one stream costs the drain once per
// range: r02n group line, 4 launches 7.38 ms vs one 6.80 ms).  fork: aux after everything issued
// on s; join: s after everything issued on aux.
hipStream_t range_stream(const pgh_ctx* c, hipStream_t s, int k) {
    return (k & 1) ? c->aux : s;
}
int fork_aux(pgh_ctx* c, hipStream_t s) {
    CK(c, hipEventRecord(c->aux_ev, s));
    CK(c, hipStreamWaitEvent(c->aux, c->aux_ev, 0));
    return PGH_OK;
}
int join_aux(pgh_ctx* c, hipStream_t s) {
    CK(c, hipEventRecord(c->aux_ev, c->aux));
    CK(c, hipStreamWaitEvent(s, c->aux_ev, 0));
    return PGH_OK;
}

// Ranges of a FINAL fold pass: 1, or final_split 4-aligned ranges of the shard.
int final_ranges(const pgh_ctx* c) { return c->final_split > 1 && c->pg >= (1 << 20) ? c->final_split : 1; }
int64_t range_edge(const pgh_ctx* c, int k, int K) { return k >= K ? c->pg : (c->pg * k / K) & ~(int64_t)3; }

int take_pin_slot(pgh_ctx* c, int* slot) {
    *slot = c->pin_next;
    c->pin_next ^= 1;
    if (c->pin_used[*slot]) CK(c, hipEventSynchronize(c->pin_ev[*slot]));
    c->pre_d2h_valid = false;  // (conservative) its cells may be overwritten now
    return PGH_OK;
}

// The stream and page-locked cells of piped rings (own_d2h): at least `bytes` of cells.  Made on
// first use; grown only after every piece already on the stream has landed.
static int ensure_d2h_cells(pgh_ctx* c, size_t bytes) {
    if (!c->d2h) {  // (made with the context, primed by its warm-up; here only if that failed)
        CK(c, hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking));
        // prime the stream with a small H2D: the runtime then runs its D2H copies on an SDMA engine
        // (an unprimed stream's D2H went to blit kernels that share the CUs with the fold, r05k/-r05x/)
        void* d = nullptr;
        CK(c, hipMalloc(&d, 64));
        const hipError_t e1 = hipMemcpyAsync(d, c->h_pin[0], 64, hipMemcpyHostToDevice, c->d2h);
        const hipError_t e2 = e1 == hipSuccess ? hipStreamSynchronize(c->d2h) : e1;
        (void)hipFree(d);
        CK(c, e2);
    }
    if (c->d2h_cap >= bytes) return PGH_OK;
    CK(c, hipStreamSynchronize(c->d2h));
    if (c->h_d2h) (void)hipHostFree(c->h_d2h);
    c->h_d2h = nullptr;
    c->d2h_cap = 0;
    if (hipHostMalloc((void**)&c->h_d2h, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, PGH_E_OOM, "page-locked D2H cells of %zu bytes failed", bytes);
    }
    c->d2h_cap = bytes;
    return PGH_OK;
}

int d2h_ring_begin(pgh_ctx* c, pgh_ctx::D2HRing* r, const uint8_t* src, size_t total, hipStream_t s, bool piped,
                   bool may_wait) {
    *r = pgh_ctx::D2HRing{};
    r->src = src;
    r->total = total;
    r->piped = piped;
    if (piped && c->own_d2h) {  // up to D2H_OWN_CELLS pieces in flight, none of the staging slots held
        r->piece = D2H_PIECE;
        r->n_pieces = (total + r->piece - 1) / r->piece;
        RC(ensure_d2h_cells(c, std::min(r->n_pieces, D2H_OWN_CELLS) * r->piece));
        r->base = c->h_d2h;
        r->cells = c->d2h_cap / r->piece;
        r->per_slot = r->cells;
        r->s = c->d2h;
        while (c->d2h_ev.size() < std::min(r->cells, r->n_pieces)) {
            hipEvent_t e = nullptr;
            CK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->d2h_ev.push_back(e);
        }
        return PGH_OK;
    }
    r->s = piped ? c->copy : s;
    r->piece = std::min(c->pin_slot, D2H_PIECE);
    r->per_slot = c->pin_slot / r->piece;  // >= 1 (pin_slot >= 4096)
    // an earlier staged ingest may still read a slot: use the free ones, wait only if neither is
    for (int k = 0; k < 2; ++k) {
        if (c->pin_used[k]) {
            const hipError_t q = hipEventQuery(c->pin_ev[k]);
            if (q == hipErrorNotReady) continue;
            CK(c, q);
            c->pin_used[k] = false;
        }
        r->free_slot[r->n_free++] = k;
    }
    if (r->n_free == 0 && !may_wait) return PGH_OK;
    if (r->n_free == 0) {
        for (int k = 0; k < 2; ++k) {
            CK(c, hipEventSynchronize(c->pin_ev[k]));
            c->pin_used[k] = false;
            r->free_slot[k] = k;
        }
        r->n_free = 2;
    }
    r->cells = (size_t)r->n_free * r->per_slot;  // ring cells, one piece each
    r->n_pieces = (total + r->piece - 1) / r->piece;
    while (c->d2h_ev.size() < std::min(r->cells, r->n_pieces)) {
        hipEvent_t e = nullptr;
        CK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->d2h_ev.push_back(e);
    }
    return PGH_OK;
}

static uint8_t* d2h_cell(const pgh_ctx* c, const pgh_ctx::D2HRing& r, size_t j) {
    if (r.base) return r.base + (j % r.cells) * r.piece;
    return c->h_pin[r.free_slot[(j % r.cells) / r.per_slot]] + (j % r.per_slot) * r.piece;
}

// Piece j of a piped ring: have all the fold ranges its floats come from finished?  (wait: block
// until they have.)  Marks may come from two streams (a split resident FINAL pass): every mark
// overlapping the piece is checked.
static int d2h_piece_ready(pgh_ctx* c, const pgh_ctx::D2HRing& r, size_t j, bool wait, bool* ready) {
    *ready = true;
    if (!r.piped) return PGH_OK;
    const size_t off = j * r.piece, len = std::min(r.piece, r.total - off);
    const int64_t first = (int64_t)(off / 4), last = (int64_t)((off + len + 3) / 4);
    int64_t start = 0;
    for (auto& m : c->final_marks) {
        if (start >= last) break;
        if (m.end > first) {
            if (wait) {
                CK(c, hipEventSynchronize(m.ev));
            } else {
                const hipError_t q = hipEventQuery(m.ev);
                if (q == hipErrorNotReady) { *ready = false; return PGH_OK; }
                CK(c, q);
            }
        }
        start = m.end;
    }
    return PGH_OK;
}

static int d2h_issue(pgh_ctx* c, pgh_ctx::D2HRing* r) {
    const size_t j = r->queued, off = j * r->piece, len = std::min(r->piece, r->total - off);
    CK(c, hipMemcpyAsync(d2h_cell(c, *r, j), r->src + off, len, hipMemcpyDeviceToHost, r->s));
    c->st.d2h_bytes_total += len;
    CK(c, hipEventRecord(c->d2h_ev[j % r->cells], r->s));
    ++r->queued;
    return PGH_OK;
}

int d2h_issue_ready(pgh_ctx* c, pgh_ctx::D2HRing* r) {
    while (r->queued < r->n_pieces && r->queued < r->done + r->cells) {
        bool ok = false;
        RC(d2h_piece_ready(c, *r, r->queued, false, &ok));
        if (!ok) break;
        RC(d2h_issue(c, r));
    }
    return PGH_OK;
}

// HBM bytes at `src` (after the work already on stream `s`) -> host pieces, through the pinned
// ring, in pieces of at most D2H_PIECE; the host copies piece k out as soon as it has landed while
// the later pieces' DMAs run.  `overlap`, if given, is host work run while the first DMA is in
// flight (the checkpoint template's framing copy).
//   Not piped: every piece that fits the ring (2 x 128 MiB by default) is queued at once on `s`.
//   marks (src is the resident checkpoint and its last fold left range marks): the pieces go on the
// copy stream, each issued once the host sees the ranges that wrote it finished (hipEventQuery /
// hipEventSynchronize), the first before the framing copy.  Issued that way the D2H runs on the
// SDMA engines beside the fold: queued with device-side waits on the marks, the runtime ran them as
// blit kernels (__amd_rocclr_copyBuffer) -- on the copy stream only after a stall, on any other
// stream always -- and each blit held the fold range beside it to a quarter of its speed (48 ->
// 182 us, profiles/r05d/, r05k/-r05m/).  The FINAL pass of a report-time close starts this itself
// (pre_d2h), issuing the pieces whose ranges are done while it issues the rest.
int stage_d2h_pieces(pgh_ctx* c, const uint8_t* src, const std::vector<OutPiece>& pieces, hipStream_t s,
                     const std::function<void()>& overlap, bool marks) {
    size_t total = 0;
    for (auto& p : pieces) total += p.n;
    if (total == 0) return PGH_OK;
    const bool piped = marks && !c->final_marks.empty();
    pgh_ctx::D2HRing r;
    if (piped && c->pre_d2h_valid && c->pre_d2h.src == src && c->pre_d2h.total == total) {
        r = c->pre_d2h;  // started by the FINAL pass (its slots marked busy until now)
    } else {
        RC(d2h_ring_begin(c, &r, src, total, s, piped));
    }
    c->pre_d2h_valid = false;
    auto copy_out = [&](size_t j) {
        const size_t off = j * r.piece, len = std::min(r.piece, total - off);
        scatter_out(d2h_cell(c, r, j), off, len, pieces, *c->pool_copy);
    };
    const int rc = [&]() -> int {  // (on failure: drain the stream below)
        if (!piped) {
            while (r.queued < r.n_pieces && r.queued < r.cells) RC(d2h_issue(c, &r));
            if (overlap) overlap();
            for (; r.done < r.n_pieces; ++r.done) {
                CK(c, hipEventSynchronize(c->d2h_ev[r.done % r.cells]));
                copy_out(r.done);
                if (r.queued < r.n_pieces) RC(d2h_issue(c, &r));  // into the cell just copied out
            }
        } else {
            RC(d2h_issue_ready(c, &r));
            if (r.queued == r.done) {  // the first piece before the framing copy
                bool ok = false;
                RC(d2h_piece_ready(c, r, r.queued, true, &ok));
                RC(d2h_issue(c, &r));
            }
            if (overlap) overlap();
            while (r.done < r.n_pieces) {
                RC(d2h_issue_ready(c, &r));  // whatever finished, before a copy-out takes the thread
                if (r.done < r.queued) {
                    const hipError_t q = hipEventQuery(c->d2h_ev[r.done % r.cells]);
                    if (q == hipSuccess) {
                        copy_out(r.done++);
                        continue;
                    }
                    if (q != hipErrorNotReady) CK(c, q);
                    std::this_thread::yield();
                } else {  // nothing in flight: wait for the next piece's ranges
                    bool ok = false;
                    RC(d2h_piece_ready(c, r, r.queued, true, &ok));
                    RC(d2h_issue(c, &r));
                }
            }
        }
        return PGH_OK;
    }();
    if (rc != PGH_OK) (void)hipStreamSynchronize(r.s);  // no piece may still land in a slot handed out later
    for (int k = 0; k < r.n_free; ++k) c->pin_used[r.free_slot[k]] = false;  // every piece landed
    return rc;
}

// The shard's slice of every tensor payload of a State message, as byte ranges of the message.
int state_shard_spans(pgh_ctx* c, const uint8_t* pb, size_t n, std::vector<std::pair<size_t, size_t>>* out,
                      const char* what) {
    std::vector<pgh_state::Span> spans;
    std::string msg;
    int rc = pgh_state::scan(pb, n, &spans, &msg);
    if (rc) return fail(c, rc, "%s State: %s", what, msg.c_str());
    if (spans.size() != c->numel.size())
        return fail(c, PGH_E_PARSE, "%s State holds %zu tensors, layout has %zu", what, spans.size(), c->numel.size());
    out->clear();
    int64_t off = 0;
    for (size_t t = 0; t < spans.size(); ++t) {
        if (spans[t].count != c->numel[t])
            return fail(c, PGH_E_PARSE, "%s tensor %zu holds %lld floats, layout %lld", what, t,
                        (long long)spans[t].count, (long long)c->numel[t]);
        const int64_t a = std::max(off, c->lo), b = std::min(off + spans[t].count, c->hi);
        if (a < b) out->push_back({spans[t].offset + 4 * (size_t)(a - off), 4 * (size_t)(b - a)});
        off += spans[t].count;
    }
    return PGH_OK;
}

// Stream `s` waits for every ingest copy / synthetic fill / varint decode issued so far.
int order_after_ingest(pgh_ctx* c, hipStream_t s) {
    CK(c, hipEventRecord(c->copy_done, c->copy));
    CK(c, hipStreamWaitEvent(s, c->copy_done, 0));
    if (c->dec_last) CK(c, hipStreamWaitEvent(s, c->dec_last, 0));
    return PGH_OK;
}

void release_slot_fold_events(pgh_ctx* c) {
    for (auto& fe : c->slab_evs) c->fold_ev_pool.push_back(fe.second);
    c->slab_evs.clear();
    for (auto& r : c->slot_ring) c->fold_ev_pool.push_back(r.second);
    c->slot_ring.clear();
    std::fill(c->slot_read_seq.begin(), c->slot_read_seq.end(), 0);
}

hipEvent_t take_fold_event(pgh_ctx* c) {
    hipEvent_t ev = nullptr;
    if (!c->fold_ev_pool.empty()) { ev = c->fold_ev_pool.back(); c->fold_ev_pool.pop_back(); }
    else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
    return ev;
}

// A fold reading every slab row was issued on stream s.
int record_slab_fold(pgh_ctx* c, hipStream_t s) {
    hipEvent_t ev = nullptr;
    for (auto& fe : c->slab_evs)
        if (fe.first == s) ev = fe.second;
    if (!ev) {
        if (!(ev = take_fold_event(c))) return fail(c, PGH_E_HIP, "hipEventCreate failed");
        c->slab_evs.push_back({s, ev});
    }
    CK(c, hipEventRecord(ev, s));
    return PGH_OK;
}

// A slot fold reading `slots` was issued on c->stream.
int record_slot_fold(pgh_ctx* c, const int32_t* slots, int n) {
    hipEvent_t ev = take_fold_event(c);
    if (!ev) return fail(c, PGH_E_HIP, "hipEventCreate failed");
    CK(c, hipEventRecord(ev, c->stream));
    const int64_t seq = ++c->slot_seq;
    c->slot_ring.push_back({seq, ev});
    for (int k = 0; k < n; ++k) c->slot_read_seq[(size_t)slots[k]] = seq;
    while (c->slot_ring.size() > 64) {  // an older fold is done when a newer one on its stream is
        c->fold_ev_pool.push_back(c->slot_ring.front().second);
        c->slot_ring.pop_front();
    }
    return PGH_OK;
}

// RESIDENT: before the copy stream overwrites `slot`, it waits for the folds that may still read it.
int order_slot_overwrite(pgh_ctx* c, int slot) {
    for (auto& fe : c->slab_evs) CK(c, hipStreamWaitEvent(c->copy, fe.second, 0));
    for (auto& fe : c->slab_evs) c->fold_ev_pool.push_back(fe.second);
    c->slab_evs.clear();
    const int64_t seq = c->slot_read_seq[(size_t)slot];
    if (seq == 0 || c->slot_ring.empty()) return PGH_OK;
    hipEvent_t ev = c->slot_ring.back().second;
    for (auto& r : c->slot_ring)
        if (r.first >= seq) { ev = r.second; break; }  // that fold, or a later one on c->stream
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return PGH_OK;
    if (q != hipErrorNotReady) return fail(c, PGH_E_HIP, "hipEventQuery failed: %s", hipGetErrorString(q));
    (void)hipGetLastError();
    CK(c, hipStreamWaitEvent(c->copy, ev, 0));
    return PGH_OK;
}

// Before the copy stream overwrites a slot, it waits for every fold issued so far (the last one
// on each stream that ran folds).
int order_before_overwrite(pgh_ctx* c) {
    for (auto& fe : c->fold_evs) CK(c, hipStreamWaitEvent(c->copy, fe.second, 0));
    for (auto& fe : c->fold_evs) c->fold_ev_pool.push_back(fe.second);
    c->fold_evs.clear();
    return PGH_OK;
}

// Remember the fold just issued on stream s.
int record_fold(pgh_ctx* c, hipStream_t s) {
    hipEvent_t ev = nullptr;
    for (auto& fe : c->fold_evs)
        if (fe.first == s) ev = fe.second;
    if (!ev) {
        if (!c->fold_ev_pool.empty()) { ev = c->fold_ev_pool.back(); c->fold_ev_pool.pop_back(); }
        else CK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->fold_evs.push_back({s, ev});
    }
    CK(c, hipEventRecord(ev, s));
    return PGH_OK;
}

void clear_marks(pgh_ctx* c) {
    for (auto& m : c->marks) c->mark_pool.push_back(m.ev);
    c->marks.clear();
}

// STREAM: the slots of clients up to `last_client` held clients up to last_client - R before;
// the copy stream waits for the fold that consumed those.
int order_stream_overwrite(pgh_ctx* c, int64_t last_client) {
    const int64_t prev = last_client - c->slots;
    while (!c->marks.empty() && c->marks.front().upto <= c->folded - c->slots) {
        c->mark_pool.push_back(c->marks.front().ev);  // no future claim needs it
        c->marks.pop_front();
    }
    if (prev < 0) return PGH_OK;  // first pass over the ring (pgh_stream_begin drained older folds)
    for (auto& m : c->marks)
        if (m.upto > prev) {
            CK(c, hipStreamWaitEvent(c->copy, m.ev, 0));
            return PGH_OK;
        }
    return order_before_overwrite(c);
}

int record_mark(pgh_ctx* c, hipStream_t s, int64_t upto) {
    hipEvent_t e = nullptr;
    if (!c->mark_pool.empty()) { e = c->mark_pool.back(); c->mark_pool.pop_back(); }
    else CK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(c, hipEventRecord(e, s));
    c->marks.push_back({e, upto});
    return PGH_OK;
}

int sync_weights(pgh_ctx* c, hipStream_t s) {
    if (c->weights_on_device || c->weights.empty()) return PGH_OK;
    if (c->weights.size() > c->w_cap) {
        (void)hipFree(c->d_w);
        c->d_w = nullptr;
        c->w_cap = 0;
        if (hipMalloc((void**)&c->d_w, sizeof(float) * c->weights.size()) != hipSuccess) {
            (void)hipGetLastError();
            return fail(c, PGH_E_OOM, "weight vector allocation failed");
        }
        c->w_cap = c->weights.size();
    }
    CK(c, hipMemcpyAsync(c->d_w, c->weights.data(), sizeof(float) * c->weights.size(), hipMemcpyHostToDevice, s));
    CK(c, hipStreamSynchronize(s));  // c->weights may change after return
    c->weights_on_device = true;
    return PGH_OK;
}

// Reciprocal table covering clients [0, n) for the iterative fold's division (div_by_count in
// pgh_kernels.hip).  Grows geometrically; the upload is ordered before stream `s`'s next fold.
int ensure_recips(pgh_ctx* c, int64_t n, hipStream_t s) {
    if (n <= c->rec_cap) return PGH_OK;
    const int64_t cap = std::max<int64_t>({n, 2 * c->rec_cap, 4096});
    std::vector<double> h((size_t)cap);
    for (int64_t k = 0; k < cap; ++k) h[(size_t)k] = 1.0 / (double)(float)(k + 1);  // y as the plan sees it
    double* d = nullptr;
    if (hipMalloc((void**)&d, sizeof(double) * (size_t)cap) != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, PGH_E_OOM, "reciprocal table allocation failed");
    }
    CK(c, hipMemcpyAsync(d, h.data(), sizeof(double) * (size_t)cap, hipMemcpyHostToDevice, s));
    CK(c, hipStreamSynchronize(s));  // h is freed on return
    if (c->d_rec) c->rec_old.push_back(c->d_rec);
    c->d_rec = d;
    c->rec_cap = cap;
    return PGH_OK;
}

int fixed_point_divisor(pgh_ctx* c, int base, int prec, float* div) {
    if (base < 2 || prec < 0 || prec > 18) return fail(c, PGH_E_ARG, "bad fixed-point base %d / precision %d", base, prec);
    long double scale = 1;
    for (int k = 0; k < prec; ++k) scale *= base;
    if (scale > 9.2e18L) return fail(c, PGH_E_ARG, "base**prec overflows int64");
    *div = (float)(int64_t)scale;  // python int base**prec, promoted to float32 by the division
    return PGH_OK;
}

float weight_total(const std::vector<float>& w, int64_t n) {  // left fold, float32
    float t = w[0];
    for (int64_t k = 1; k < n; ++k) t = t + w[k];
    return t;
}

// Fold slots holding clients [c0, c0 + n) (slot order may wrap) into the running state.
// FIRST when c0 == 0; FINAL writes out (fedavg: ckpt - avg; secagg: sum/dec) instead of the state.
int fold_run(pgh_ctx* c, int kind, int64_t c0, int64_t n, bool final, const FinalArgs& fa, hipStream_t s) {
    RC(order_after_ingest(c, s));
    if (kind == PGH_WEIGHTED_MEAN && n > 0) {
        if ((int64_t)c->weights.size() < c0 + n)
            return fail(c, PGH_E_STATE, "weighted mean: %zu weights for %lld clients", c->weights.size(),
                        (long long)(c0 + n));
        RC(sync_weights(c, s));
    }
    if (kind == PGH_ITERATIVE_MEAN && n > 0) RC(ensure_recips(c, c0 + n, s));
    const int R = c->slots;
    const int64_t off = fa.off;
    const int64_t len = fa.len < 0 ? c->pg - off : fa.len;
    if (off < 0 || (off & 3) || len <= 0 || off + len > c->pg)
        return fail(c, PGH_E_ARG, "param range [%lld,+%lld) outside the shard or not 4-aligned", (long long)off,
                    (long long)len);
    int64_t done = 0;
    do {
        const int slot = (int)((c0 + done) % R);
        const int64_t seg = std::min<int64_t>(n - done, (int64_t)(R - slot));
        const bool first = (c0 + done == 0);
        const bool last = (done + seg == n);
        const int flags = (first ? pgh::FL_FIRST : 0) | (final && last ? pgh::FL_FINAL : 0);
        const uint64_t pg = (uint64_t)len;
        if (kind == KIND_SECAGG) {
            pgh::SecaggArgs a{};
            a.shares = (const int64_t*)slot_row(c, slot, 0);
            a.map = slab_map(c);
            a.map.off = off;
            a.n_rows = (int)(seg * c->parties);
            a.p = len;
            a.acc = c->d_uacc + off;
            a.sum_out = fa.sum ? fa.sum + off : nullptr;
            a.dec_out = fa.dec ? fa.dec + off : nullptr;
            a.divisor = fa.divisor;
            a.flags = flags;
            a.variant = c->variant;
            const uint64_t bytes = 8ull * (uint64_t)a.n_rows * pg + (first ? 0 : 8 * pg) +
                                   ((flags & pgh::FL_FINAL) ? (fa.sum ? 8 * pg : 0) + (fa.dec ? 4 * pg : 0) : 8 * pg);
            RC(timed_launch(c, s, bytes, [&] { return pgh::launch_secagg(a, s); }));
        } else {
            pgh::FedavgArgs a{};
            a.diffs = (const float*)slot_row(c, slot, 0);
            a.map = slab_map(c);
            a.map.off = off;
            a.n_rows = (int)seg;
            a.client0 = c0 + done;
            a.p = len;
            a.weights = c->d_w ? c->d_w + (c0 + done) : nullptr;
            a.recips = c->d_rec ? c->d_rec + (c0 + done) : nullptr;
            a.acc = c->d_acc + off;
            a.ckpt = fa.ckpt ? fa.ckpt + off : nullptr;
            a.out = fa.out ? fa.out + off : nullptr;
            a.divisor = fa.divisor;
            a.flags = flags;
            a.mode = kind;
            a.variant = c->variant;
            const uint64_t bytes = 4ull * (uint64_t)seg * pg + (first ? 0 : 4 * pg) +
                                   ((flags & pgh::FL_FINAL) ? 8 * pg : 4 * pg);
            RC(timed_launch(c, s, bytes, [&] { return pgh::launch_fedavg(a, s); }));
        }
        done += seg;
    } while (done < n);
    RC(record_fold(c, s));
    return record_slab_fold(c, s);
}

// Length of the run of ingested clients starting at `from` (slot ring order).
int64_t ready_run(pgh_ctx* c, int64_t from) {
    int64_t n = 0;
    while (n < c->slots && c->slot_client[(size_t)((from + n) % c->slots)] == from + n) ++n;
    return n;
}

// Every ingested client must belong to the contiguous run starting at `from`.
int check_no_gaps(pgh_ctx* c, int64_t from, int64_t run) {
    for (int s = 0; s < c->slots; ++s) {
        const int64_t k = c->slot_client[(size_t)s];
        if (k >= 0 && (k < from || k >= from + run))
            return fail(c, PGH_E_STATE, "client %lld is missing but client %lld was ingested",
                        (long long)(from + run), (long long)k);
    }
    return PGH_OK;
}

// STREAM: fold the ready run when it reaches the batch size (or always, when forced).
int maybe_fold(pgh_ctx* c, bool force) {
    const int64_t run = ready_run(c, c->folded);
    if (run == 0 || (!force && run < c->fold_batch)) return PGH_OK;
    RC(fold_run(c, c->kind, c->folded, run, false, FinalArgs{}, c->stream));
    for (int64_t k = 0; k < run; ++k) c->slot_client[(size_t)((c->folded + k) % c->slots)] = -1;
    c->folded += run;
    c->st.n_folded = c->folded;
    return record_mark(c, c->stream, c->folded);
}

// Claim the slot for `client` (both modes) before bytes are written to it.
int claim_slot(pgh_ctx* c, int64_t client, int* slot_out) {
    if (client < 0) return fail(c, PGH_E_ARG, "negative client index");
    if (!c->streaming) {
        if (client >= c->slots)
            return fail(c, PGH_E_ARG, "client %lld outside slab capacity %d", (long long)client, c->slots);
        RC(order_slot_overwrite(c, (int)client));  // a fold issued earlier may still read the slot
        *slot_out = (int)client;
        return PGH_OK;
    }
    if (client < c->folded) return fail(c, PGH_E_STATE, "client %lld was already folded", (long long)client);
    const int slot = (int)(client % c->slots);
    const int64_t held = c->slot_client[(size_t)slot];
    if (held >= 0 && held != client)
        return fail(c, PGH_E_STATE, "ring full: slot %d still holds unfolded client %lld (fold front %lld)", slot,
                    (long long)held, (long long)c->folded);
    RC(order_stream_overwrite(c, client));
    *slot_out = slot;
    return PGH_OK;
}

int mark_ingested(pgh_ctx* c, int64_t client, int slot) {
    if (c->slot_client[(size_t)slot] != client) c->st.n_clients += 1;
    c->slot_client[(size_t)slot] = client;
    return c->streaming ? maybe_fold(c, false) : PGH_OK;
}

// RESIDENT: clients [0, n) all present, nothing else.
int resident_count(pgh_ctx* c, int64_t* n_out) {
    if (c->streaming) return fail(c, PGH_E_STATE, "context is streaming: finish with pgh_stream_finish*");
    int64_t n = ready_run(c, 0);
    RC(check_no_gaps(c, 0, n));
    if (n == 0) return fail(c, PGH_E_STATE, "no diffs ingested");
    *n_out = n;
    return PGH_OK;
}

int fedavg_divisor(pgh_ctx* c, int mode, int64_t n, float* div) {
    if (mode == PGH_WEIGHTED_MEAN) {
        if ((int64_t)c->weights.size() < n)
            return fail(c, PGH_E_STATE, "weighted mean needs %lld weights, have %zu", (long long)n, c->weights.size());
        const float t = weight_total(c->weights, n);
        if (!(t != 0.f)) return fail(c, PGH_E_ARG, "sum of weights is zero");
        *div = t;
    } else {
        *div = (float)n;  // th.div(sum, len(diffs)), cycle_manager.py:288
    }
    return PGH_OK;
}


// caller stream `cs` -> context stream ordering, and back
int join_in(pgh_ctx* c, hipStream_t cs) {
    if (cs == c->stream) return PGH_OK;
    CK(c, hipEventRecord(c->xsync, cs));
    CK(c, hipStreamWaitEvent(c->stream, c->xsync, 0));
    return PGH_OK;
}
int join_out(pgh_ctx* c, hipStream_t cs) {
    if (cs == c->stream) return PGH_OK;
    CK(c, hipEventRecord(c->xsync, c->stream));
    CK(c, hipStreamWaitEvent(cs, c->xsync, 0));
    return PGH_OK;
}

// ---- page-locked blocks whose DMAs may outlive the ingest call -------------------------------------
// pgh_host_async marks a pgh_host_alloc block: an ingest from it then returns once the DMA is queued
// (not done), and records the DMA's event here; pgh_host_wait(p, n) waits for every DMA still reading
// [p, p + n) (any context, any GPU) before the owner reuses or frees the block.  Unmarked page-locked
// memory keeps the synchronous contract (the call waits for its copies).
struct HostDma { uintptr_t lo, hi; hipEvent_t ev; };
std::mutex g_host_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_async_blocks;  // [lo, hi)
std::vector<HostDma> g_host_dmas;

bool host_async(const void* p, size_t n) {
    const uintptr_t a = (uintptr_t)p, b = a + n;
    std::lock_guard<std::mutex> lk(g_host_mu);
    for (auto& r : g_async_blocks)
        if (a >= r.first && b <= r.second) return true;
    return false;
}

// Record that a DMA reading [p, p + n) was queued on stream s (the event is recorded here).
int host_dma_queued(pgh_ctx* c, const void* p, size_t n, hipStream_t s) {
    hipEvent_t ev = nullptr;
    CK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const hipError_t e = hipEventRecord(ev, s);
    if (e != hipSuccess) {
        (void)hipEventDestroy(ev);
        return fail(c, PGH_E_HIP, "hipEventRecord failed: %s", hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> lk(g_host_mu);
    // forget DMAs that have finished (a block held elsewhere for long would otherwise collect them)
    auto keep = g_host_dmas.begin();
    for (auto& d : g_host_dmas) {
        if (hipEventQuery(d.ev) == hipSuccess) (void)hipEventDestroy(d.ev);
        else *keep++ = d;
    }
    g_host_dmas.erase(keep, g_host_dmas.end());
    (void)hipGetLastError();  // hipErrorNotReady from the queries above
    g_host_dmas.push_back({(uintptr_t)p, (uintptr_t)p + n, ev});
    return PGH_OK;
}

}  // namespace pgh_detail

using namespace pgh_detail;

extern "C" {

int pgh_abi_version(void) { return PGH_ABI_VERSION; }

int pgh_device_count(int* n) {
    if (!n) return PGH_E_ARG;
    int k = 0;
    hipError_t e = hipGetDeviceCount(&k);
    if (e != hipSuccess) { *n = 0; return fail(nullptr, PGH_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e)); }
    *n = k;
    return PGH_OK;
}

const char* pgh_last_error(const pgh_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

int pgh_host_async(void* p, size_t n, int on) {
    if (!p || !n) return fail(nullptr, PGH_E_ARG, "bad block");
    if (!on) RC(pgh_host_wait(p, n));
    std::lock_guard<std::mutex> lk(g_host_mu);
    const std::pair<uintptr_t, uintptr_t> r{(uintptr_t)p, (uintptr_t)p + n};
    auto it = std::find(g_async_blocks.begin(), g_async_blocks.end(), r);
    if (on && it == g_async_blocks.end()) g_async_blocks.push_back(r);
    if (!on && it != g_async_blocks.end()) g_async_blocks.erase(it);
    return PGH_OK;
}

int pgh_host_wait(const void* p, size_t n) {
    const uintptr_t a = (uintptr_t)p, b = a + n;
    std::vector<hipEvent_t> evs;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto keep = g_host_dmas.begin();
        for (auto& d : g_host_dmas) {
            if (d.lo < b && a < d.hi) evs.push_back(d.ev);
            else *keep++ = d;
        }
        g_host_dmas.erase(keep, g_host_dmas.end());
    }
    int rc = PGH_OK;
    for (hipEvent_t ev : evs) {
        const hipError_t e = hipEventSynchronize(ev);
        if (e != hipSuccess && rc == PGH_OK) rc = fail(nullptr, PGH_E_HIP, "DMA from host buffer failed: %s",
                                                       hipGetErrorString(e));
        (void)hipEventDestroy(ev);
    }
    return rc;
}

int pgh_host_alloc(size_t bytes, void** out) {
    if (!out || !bytes) return fail(nullptr, PGH_E_ARG, "bad pinned allocation request");
    *out = nullptr;
    if (hipHostMalloc(out, bytes, hipHostMallocPortable) != hipSuccess) {  // DMA-able by every GPU of a group
        (void)hipGetLastError();
        *out = nullptr;
        return fail(nullptr, PGH_E_OOM, "pinned host allocation of %zu bytes failed", bytes);
    }
    return PGH_OK;
}

int pgh_host_prefault(void* p, size_t n) {
    if (!p || !n) return PGH_OK;
    const size_t per = (size_t)8 << 20;
    const int k = (int)std::min<size_t>(8, (n + per - 1) / per);
    if (k <= 1) {
        prefault_small_any((uint8_t*)p, n);
        return PGH_OK;
    }
    std::vector<std::thread> ts;
    const size_t step = (n + (size_t)k - 1) / (size_t)k;
    for (int i = 0; i < k; ++i) {
        const size_t a = (size_t)i * step, b = std::min(n, a + step);
        if (a < b) ts.emplace_back([=] { prefault_small_any((uint8_t*)p + a, b - a); });
    }
    for (auto& t : ts) t.join();
    return PGH_OK;
}

int pgh_host_free(void* p) {
    if (p) {
        size_t n = 0;
        {
            std::lock_guard<std::mutex> lk(g_host_mu);
            for (auto it = g_async_blocks.begin(); it != g_async_blocks.end(); ++it)
                if (it->first == (uintptr_t)p) {
                    n = it->second - it->first;
                    g_async_blocks.erase(it);
                    break;
                }
        }
        if (n) (void)pgh_host_wait(p, n);  // a DMA from the block may still be running
    }
    if (p && hipHostFree(p) != hipSuccess) return fail(nullptr, PGH_E_HIP, "hipHostFree failed");
    return PGH_OK;
}

int pgh_create(int device, size_t pinned_bytes, pgh_ctx** out) {
    if (!out) return fail(nullptr, PGH_E_ARG, "out is NULL");
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) return fail(nullptr, PGH_E_HIP, "no HIP device: %s", hipGetErrorString(e));
    if (device < 0 || device >= ndev) return fail(nullptr, PGH_E_ARG, "device %d out of range [0,%d)", device, ndev);
    auto* c = new pgh_ctx();
    c->device = device;
    DeviceGuard g(device);
    if (pinned_bytes == 0) pinned_bytes = 256ull << 20;
    c->pin_slot = (pinned_bytes / 2) & ~(size_t)4095;
    if (c->pin_slot < 4096) c->pin_slot = 4096;
    c->copy_threads = std::min(16, pgh_int::usable_cpus());
    if (const char* e = std::getenv("PGH_COPY_THREADS")) c->copy_threads = std::max(1, std::atoi(e));
    {
        const char* nu = std::getenv("PGH_NUMA");
        if (!nu || std::atoi(nu) != 0) c->local_cpus = gpu_local_cpus(device);
    }
    c->pool_copy.reset(new CopyPool(c->copy_threads, c->local_cpus));
    if (const char* e = std::getenv("PGH_PINNED_GATHER")) c->pinned_gather = std::atoi(e) != 0;
    if (const char* e = std::getenv("PGH_BLOCK_BYTES")) c->block_bytes = (size_t)std::max(0LL, std::atoll(e));
    if (const char* e = std::getenv("PGH_FINAL_RANGES")) c->final_split = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("PGH_D2H_STREAM")) c->d2h_mode = std::max(0, std::min(1, std::atoi(e)));
    c->own_d2h = c->d2h_mode > 0;
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&c->copy_done, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->xsync, hipEventDisableTiming) == hipSuccess &&
              hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&c->aux_ev, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->pin_ev[0], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->pin_ev[1], hipEventDisableTiming) == hipSuccess &&
              (!c->own_d2h || hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking) == hipSuccess);
    if (!ok) { pgh_destroy(c); return fail(nullptr, PGH_E_HIP, "stream/event creation failed"); }
    {
        // the pinned ring on the GPU's socket: allocated by a thread bound there, pages placed by
        // its (local) memory policy
        bool pin_ok = true;
        auto alloc = [&] {
            bind_thread(c->local_cpus);
            const unsigned flags = c->local_cpus.empty() ? hipHostMallocDefault : hipHostMallocNumaUser;
            for (int k = 0; k < 2 && pin_ok; ++k) {
                if (hipHostMalloc((void**)&c->h_pin[k], c->pin_slot, flags) == hipSuccess) continue;
                (void)hipGetLastError();
                // a placement the runtime refuses is not worth failing the context for
                if (flags != hipHostMallocDefault &&
                    hipHostMalloc((void**)&c->h_pin[k], c->pin_slot, hipHostMallocDefault) == hipSuccess)
                    continue;
                (void)hipGetLastError();
                c->h_pin[k] = nullptr;
                pin_ok = false;
            }
        };
        if (c->local_cpus.empty()) alloc();
        else std::thread([&] { DeviceGuard g2(device); alloc(); }).join();
        if (!pin_ok) {
            pgh_destroy(c);
            return fail(nullptr, PGH_E_OOM, "pinned host allocation of %zu bytes failed", c->pin_slot);
        }
    }
    // Warm-up (PGH_WARMUP=0 skips it): the first kernel launch loads the code object and the first
    // copies set up the runtime's copy engines (the first ~1 MB H2D from the pinned ring took 8.3 ms
    // of host time, r01ao) -- ~11 ms that would otherwise land on the node's first cycle close
    // (profiles/r01am).  One small launch plus an H2D and a D2H of up to 2 MiB on the two streams.
    const char* wu = std::getenv("PGH_WARMUP");
    if (!wu || std::atoi(wu) != 0) {
        const int64_t n = (int64_t)std::min(c->pin_slot, (size_t)2 << 20) / 8;  // int64 values
        void* d = nullptr;
        ok = hipMalloc(&d, 12 * n) == hipSuccess;
        if (ok) {
            int64_t* d_sum = (int64_t*)d;
            float* d_dec = (float*)((uint8_t*)d + 8 * n);
            std::memset(c->h_pin[0], 0, 8 * n);
            ok = hipMemcpyAsync(d_sum, c->h_pin[0], 8 * n, hipMemcpyHostToDevice, c->copy) == hipSuccess &&
                 hipStreamSynchronize(c->copy) == hipSuccess &&
                 (!c->d2h || (hipMemcpyAsync(d_sum, c->h_pin[0], 8 * n, hipMemcpyHostToDevice, c->d2h) == hipSuccess &&
                              hipStreamSynchronize(c->d2h) == hipSuccess)) &&
                 pgh::launch_secagg_decode(d_sum, d_dec, n, 1.0f, c->stream) == hipSuccess &&
                 hipMemcpyAsync(c->h_pin[1], d_sum, 8 * n, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
                 hipStreamSynchronize(c->stream) == hipSuccess;
            (void)hipFree(d);
        }
        if (!ok) {  // best effort: a latency optimisation must not cost the node its engine
            (void)hipGetLastError();
            (void)hipStreamSynchronize(c->copy);
            (void)hipStreamSynchronize(c->stream);
            c->warmup_skipped = true;
        }
    }
    *out = c;
    return PGH_OK;
}

void pgh_destroy(pgh_ctx* c) {
    if (!c) return;
    if (c->grp) { pgh_group_api::destroy(c); return; }
    DeviceGuard g(c->device);
    free_slab(c);
    for (auto& t : c->pending) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    clear_marks(c);
    for (auto e : c->mark_pool) (void)hipEventDestroy(e);
    (void)hipFree(c->d_rec);
    for (double* p : c->rec_old) (void)hipFree(p);
    (void)hipFree(c->d_vbytes);
    if (c->dec) (void)hipStreamSynchronize(c->dec);
    for (auto& b : c->vbuf) {
        (void)hipFree(b.bytes);
        (void)hipFree(b.tab);
        if (b.done) (void)hipEventDestroy(b.done);
    }
    if (c->dec_in) (void)hipEventDestroy(c->dec_in);
    if (c->dec) (void)hipStreamDestroy(c->dec);
    if (c->h_vtab) (void)hipHostFree(c->h_vtab);
    if (c->vtab_ev) (void)hipEventDestroy(c->vtab_ev);
    (void)hipFree(c->d_gtab);
    if (c->h_gtab) (void)hipHostFree(c->h_gtab);
    if (c->gtab_ev) (void)hipEventDestroy(c->gtab_ev);
    if (c->gdma_ev) (void)hipEventDestroy(c->gdma_ev);
    for (int k = 0; k < 2; ++k) {
        if (c->h_pin[k]) (void)hipHostFree(c->h_pin[k]);
        if (c->pin_ev[k]) (void)hipEventDestroy(c->pin_ev[k]);
    }
    if (c->d2h) (void)hipStreamSynchronize(c->d2h);
    if (c->h_d2h) (void)hipHostFree(c->h_d2h);
    if (c->d2h) (void)hipStreamDestroy(c->d2h);
    for (hipEvent_t e : {c->copy_done, c->xsync, c->aux_ev})
        if (e) (void)hipEventDestroy(e);
    for (auto e : c->fold_ev_pool) (void)hipEventDestroy(e);
    for (auto e : c->rmark_pool) (void)hipEventDestroy(e);
    for (auto e : c->d2h_ev) (void)hipEventDestroy(e);
    for (auto e : c->rng_ev) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    delete c;
}

int pgh_set_layout(pgh_ctx* c, int n_tensors, const int64_t* numel) {
    if (c && c->grp) return pgh_group_api::set_layout(c, n_tensors, numel);
    if (!c) return PGH_E_ARG;
    if (n_tensors <= 0 || !numel) return fail(c, PGH_E_ARG, "need at least one tensor");
    int64_t P = 0;
    for (int k = 0; k < n_tensors; ++k) {
        if (numel[k] < 0) return fail(c, PGH_E_ARG, "tensor %d has negative numel", k);
        P += numel[k];
    }
    if (P <= 0) return fail(c, PGH_E_ARG, "model has no parameters");
    DeviceGuard g(c->device);
    free_slab(c);
    c->numel.assign(numel, numel + n_tensors);
    c->P = P;
    c->layout = true;
    return pgh_set_shard(c, 0, P);
}

int pgh_set_shard(pgh_ctx* c, int64_t lo, int64_t hi) {
    if (c && c->grp) return pgh_group_api::set_shard(c, lo, hi);
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (lo < 0 || hi > c->P || lo >= hi)
        return fail(c, PGH_E_ARG, "shard [%lld,%lld) outside [0,%lld)", (long long)lo, (long long)hi, (long long)c->P);
    DeviceGuard g(c->device);
    free_slab(c);
    c->lo = lo;
    c->hi = hi;
    c->pg = hi - lo;
    c->pvec = std::max((c->pg + 63) & ~(int64_t)63, (c->vec_min + 63) & ~(int64_t)63);
    c->st.p_shard = c->pg;
    return PGH_OK;
}

int pgh_reserve(pgh_ctx* c, int max_clients, int dtype, int n_parties) {
    if (c && c->grp) return pgh_group_api::reserve(c, max_clients, dtype, n_parties);
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (max_clients <= 0) return fail(c, PGH_E_ARG, "max_clients must be positive");
    if (dtype != PGH_F32 && dtype != PGH_I64) return fail(c, PGH_E_ARG, "unknown dtype %d", dtype);
    if (dtype == PGH_F32) n_parties = 1;
    if (n_parties < 1) return fail(c, PGH_E_ARG, "n_parties must be >= 1");
    DeviceGuard g(c->device);
    free_slab(c);
    const size_t rows = (size_t)max_clients * (size_t)n_parties;
    slab_geometry(c->pg, esize(dtype), c->block_bytes, &c->bw, &c->nb, &c->bshift);
    c->bmask = c->bshift == 62 ? (int64_t(1) << 62) - 1 : c->bw - 1;
    c->bstride = c->nb > 1 ? (int64_t)rows * c->bw : 0;
    const size_t bytes = rows * (size_t)(c->nb * c->bw) * esize(dtype);
    if (hipMalloc(&c->d_slab, bytes) != hipSuccess) {
        c->d_slab = nullptr;
        (void)hipGetLastError();
        return fail(c, PGH_E_OOM, "slab allocation of %zu bytes (%zu rows x %lld) failed", bytes, rows,
                    (long long)(c->nb * c->bw));
    }
    c->slab_bytes = bytes;
    c->st.ld = c->bw;
    const size_t v4 = (size_t)c->pvec * 4, v8 = (size_t)c->pvec * 8;
    bool ok = hipMalloc((void**)&c->d_ckpt, v4) == hipSuccess && hipMalloc((void**)&c->d_out, v4) == hipSuccess &&
              hipMalloc((void**)&c->d_acc, v4) == hipSuccess && hipMalloc((void**)&c->d_uacc, v8) == hipSuccess &&
              hipMalloc((void**)&c->d_sum, v8) == hipSuccess && hipMalloc((void**)&c->d_dec, v4) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        free_slab(c);
        return fail(c, PGH_E_OOM, "device vector allocation failed");
    }
    c->slots = max_clients;
    c->dtype = dtype;
    c->parties = n_parties;
    c->slot_client.assign((size_t)max_clients, -1);
    c->slot_read_seq.assign((size_t)max_clients, 0);
    c->weights.clear();
    c->weights_on_device = false;
    c->st.max_clients = max_clients;
    c->st.n_clients = 0;
    c->st.n_folded = 0;
    return PGH_OK;
}

int pgh_reset(pgh_ctx* c) {
    if (c && c->grp) return pgh_group_api::reset(c);
    if (!c) return PGH_E_ARG;
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& fe : c->fold_evs) (void)hipEventSynchronize(fe.second);  // folds issued on caller streams
    for (auto& fe : c->fold_evs) c->fold_ev_pool.push_back(fe.second);
    c->fold_evs.clear();
    clear_marks(c);
    release_slot_fold_events(c);  // c->stream is idle (synchronised above)
    std::fill(c->slot_client.begin(), c->slot_client.end(), -1);
    c->weights.clear();
    c->weights_on_device = false;
    c->streaming = false;
    c->slot_mode = -1;
    c->folded = 0;
    c->st.n_clients = 0;
    c->st.n_folded = 0;
    return PGH_OK;
}

// ---- observability -------------------------------------------------------------------------------

int pgh_set_variant(pgh_ctx* c, int variant) {
    if (c && c->grp) return pgh_group_api::set_variant(c, variant);
    if (!c) return PGH_E_ARG;
    if (variant < -1 || variant > 23) return fail(c, PGH_E_ARG, "variant %d outside [-1,23]", variant);
    c->variant = variant;
    return PGH_OK;
}

int pgh_effective_variant(pgh_ctx* c, int mode) {
    if (c && c->grp) return pgh_group_api::effective_variant(c, mode);
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (c->variant >= 0) return c->variant;
    if (mode == PGH_STREAM_SECAGG) return 14;  // SECAGG_AUTO_VARIANT in pgh_kernels.hip
    if (!valid_mode(mode)) return fail(c, PGH_E_ARG, "unknown averaging mode %d", mode);
    return pgh::auto_variant(c->pg, mode);
}

int pgh_stats(pgh_ctx* c, pgh_stats_t* out) {
    if (c && c->grp) return pgh_group_api::stats(c, out);
    if (!c || !out) return PGH_E_ARG;
    DeviceGuard g(c->device);
    RC(collect_timings(c));
    *out = c->st;
    return PGH_OK;
}

int pgh_reset_stats(pgh_ctx* c) {
    if (c && c->grp) return pgh_group_api::reset_stats(c);
    if (!c) return PGH_E_ARG;
    DeviceGuard g(c->device);
    RC(collect_timings(c));
    pgh_stats_t keep = c->st;
    c->st = pgh_stats_t{};
    c->st.p_shard = keep.p_shard;
    c->st.ld = keep.ld;
    c->st.n_clients = keep.n_clients;
    c->st.max_clients = keep.max_clients;
    c->st.n_folded = keep.n_folded;
    return PGH_OK;
}

int pgh_slab(pgh_ctx* c, void** d_slab, int64_t* ld, int64_t* block_pitch) {
    if (c && c->grp) return fail(c, PGH_E_UNSUPPORTED, "%s takes device pointers, which name one GPU: call it on pgh_group_child", __func__);
    if (!c || !d_slab || !ld || !block_pitch) return PGH_E_ARG;
    *d_slab = c->d_slab;
    *ld = c->bw;
    *block_pitch = c->bstride;
    return PGH_OK;
}

int pgh_sync(pgh_ctx* c) {
    if (c && c->grp) return pgh_group_api::sync(c);
    if (!c) return PGH_E_ARG;
    DeviceGuard g(c->device);
    CK(c, hipStreamSynchronize(c->copy));
    if (c->dec) CK(c, hipStreamSynchronize(c->dec));
    CK(c, hipStreamSynchronize(c->stream));
    return PGH_OK;
}

}  // extern "C"

// ---- internals for the multi-GPU group driver (pgh_internal.h) ------------------------------------

namespace pgh_int {
int usable_cpus() {
    static const int n = [] {
        int cpus = 0;
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
        if (cpus <= 0) cpus = (int)std::max(1u, std::thread::hardware_concurrency());
        double quota = 0;
        std::ifstream v2("/sys/fs/cgroup/cpu.max");
        std::string q;
        long long per = 0;
        if (v2 >> q >> per) {
            if (q != "max" && per > 0) quota = std::atof(q.c_str()) / (double)per;
        } else {
            std::ifstream qf("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), pf("/sys/fs/cgroup/cpu/cpu.cfs_period_us");
            long long qq = 0, pp = 0;
            if ((qf >> qq) && (pf >> pp) && qq > 0 && pp > 0) quota = (double)qq / (double)pp;
        }
        if (quota >= 1 && (int)quota < cpus) cpus = (int)quota;
        return std::max(1, cpus);
    }();
    return n;
}

int fail(pgh_ctx* c, int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const int r = vfail(c, code, fmt, ap);
    va_end(ap);
    return r;
}
pgh_group* group_of(const pgh_ctx* c) { return c ? c->grp : nullptr; }
pgh_ctx* new_group_ctx(pgh_group* g, int device) {
    auto* c = new pgh_ctx();
    c->grp = g;
    c->device = device;
    return c;
}
void free_group_ctx(pgh_ctx* c) { delete c; }
int device_of(const pgh_ctx* c) { return c->device; }
hipStream_t stream_of(const pgh_ctx* c) { return c->stream; }
int set_vec_min(pgh_ctx* c, int64_t n) {
    if (n < 0) return fail(c, PGH_E_ARG, "negative vector length");
    c->vec_min = n;
    if (c->layout) c->pvec = std::max((c->pg + 63) & ~(int64_t)63, (c->vec_min + 63) & ~(int64_t)63);
    return PGH_OK;
}
int set_copy_threads(pgh_ctx* c, int n) {
    n = std::max(1, n);
    if (n == c->copy_threads && c->pool_copy) return PGH_OK;
    c->copy_threads = n;
    c->pool_copy.reset(new CopyPool(n, c->local_cpus));
    return PGH_OK;
}
int set_client_base(pgh_ctx* c, int64_t base) {
    c->client_base = base;
    return PGH_OK;
}
void* vec(pgh_ctx* c, int which) {
    switch (which) {
    case V_CKPT: return c->d_ckpt;
    case V_SUM: return c->d_sum;
    case V_DEC: return c->d_dec;
    default: return nullptr;
    }
}
int patch_payloads(pgh_ctx* c, const uint8_t* tmpl, size_t n, uint8_t* out) {
    RC(check_dtype(c, PGH_F32));
    if (!tmpl || !out) return fail(c, PGH_E_ARG, "tmpl / out is NULL");
    RC(check_ckpt(c, "pgh_ckpt_patch_state"));
    std::vector<std::pair<size_t, size_t>> spans;
    RC(state_shard_spans(c, tmpl, n, &spans, "checkpoint template"));
    DeviceGuard g(c->device);
    std::vector<OutPiece> pieces;
    for (auto& sp : spans) pieces.push_back(OutPiece{out + sp.first, sp.second});
    RC(order_after_ingest(c, c->stream));
    RC(stage_d2h_pieces(c, (const uint8_t*)c->d_ckpt, pieces, c->stream, [&] {
        if (!spans.empty()) {  // this shard's part of the (fresh) output
            const size_t a = spans.front().first, b = spans.back().first + spans.back().second;
            if (b > a) prefault_parallel(out + a, b - a, *c->pool_copy);
        }
    }, true));
    return collect_timings(c);
}
}  // namespace pgh_int
