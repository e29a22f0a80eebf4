// The single-GPU context (struct pgh_ctx) and the helpers its entry points share.  Not installed;
// the public surface is include/pgh_api.h.
//
// The context's entry points are split by what they do:
//   pgh_api.cpp     lifecycle (create / layout / reserve / reset / destroy), page-locked host blocks,
//                   observability, the shared helpers below, the group driver's internals
//   pgh_ingest.cpp  host bytes -> HBM slab rows (raw, State messages, int64 shares, synthetic)
//   pgh_reduce.cpp  RESIDENT and STREAM folds, the resident checkpoint, secagg
//   pgh_slots.cpp   report-time slot folds (the certain prefix of the close-time order)
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/pgh_api.h"
#include "pgh_internal.h"
#include "pgh_kernels.h"
#include "pgh_state.h"

namespace pgh_detail {

constexpr int KIND_SECAGG = 3;  // stream kind besides the three fedavg modes

// memcpy with non-temporal 16-byte stores for big copies into staging / output buffers (no
// read-for-ownership of the destination, which is written once and then read by the DMA engine or
// handed to the caller; r01ab).
void copy_stream(uint8_t* dst, const uint8_t* src, size_t n);
// Bind the calling thread to `cpus` (no-op when empty or refused).
void bind_thread(const std::vector<int>& cpus);
// CPUs on the GPU's own socket (its PCI device's local_cpulist) that this process may run on; empty
// when unknown.  Staging copies and pinned buffers there keep the host side of every H2D / D2H off
// the socket interconnect (a 2-socket node: GPUs 0-3 on one socket, 4-7 on the other).
std::vector<int> gpu_local_cpus(int device);

// Host copy engine: a persistent pool that splits one batch of (dst, src, n) segments evenly
// by bytes across its threads (the caller's thread takes the first share).  Used to fill and
// drain the pinned staging slots, where payload pieces are many and mostly small.
class CopyPool {
  public:
    struct Seg {
        uint8_t* dst;
        const uint8_t* src;
        size_t n;
    };
    explicit CopyPool(int threads, std::vector<int> cpus = {}) : nthreads_(std::max(1, threads)) {
        for (int t = 1; t < nthreads_; ++t)
            workers_.emplace_back([this, t, cpus] {
                bind_thread(cpus);
                loop(t);
            });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    int threads() const { return nthreads_; }
    void run(const std::vector<Seg>& segs) {
        size_t total = 0;
        for (auto& sg : segs) total += sg.n;
        if (total < (4u << 20) || nthreads_ == 1) { copy_range(segs, 0, total); return; }
        {
            std::lock_guard<std::mutex> lk(m_);
            segs_ = &segs;
            total_ = total;
            pending_ = nthreads_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        copy_range(segs, 0, share(total, 0));
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [this] { return pending_ == 0; });
        segs_ = nullptr;
    }

    // f(i) for every i in [0, n), items split into contiguous runs over the threads (the caller's
    // thread takes the first run).  Small jobs stay on the caller's thread.
    void run_items(int n, bool parallel, const std::function<void(int)>& f) {
        if (!parallel || nthreads_ == 1 || n < 2) { for (int i = 0; i < n; ++i) f(i); return; }
        const int per = (n + nthreads_ - 1) / nthreads_;
        std::function<void(int)> job = [&](int t) {
            for (int i = t * per; i < std::min(n, (t + 1) * per); ++i) f(i);
        };
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &job;
            pending_ = nthreads_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        job(0);
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

  private:
    size_t share(size_t total, int t) const {  // [begin, end) of thread t, 4 KiB granules
        const size_t per = ((total + nthreads_ - 1) / nthreads_ + 4095) & ~(size_t)4095;
        return std::min(total, per * (size_t)(t + 1));
    }
    static void copy_range(const std::vector<Seg>& segs, size_t a, size_t b) {
        size_t base = 0;
        for (auto& sg : segs) {
            const size_t lo = std::max(a, base), hi = std::min(b, base + sg.n);
            if (lo < hi) copy_stream(sg.dst + (lo - base), sg.src + (lo - base), hi - lo);
            base += sg.n;
            if (base >= b) break;
        }
    }
    void loop(int t) {
        uint64_t seen = 0;
        for (;;) {
            const std::vector<Seg>* segs;
            const std::function<void(int)>* fn;
            size_t total;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                segs = segs_;
                fn = fn_;
                total = total_;
            }
            if (fn) {
                (*fn)(t);
            } else {
                const size_t a = t == 0 ? 0 : share(total, t - 1);
                copy_range(*segs, std::min(a, total), share(total, t));
            }
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_cv_.notify_one();
        }
    }
    int nthreads_;
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    const std::vector<Seg>* segs_ = nullptr;
    const std::function<void(int)>* fn_ = nullptr;
    size_t total_ = 0;
    int pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace pgh_detail

struct pgh_ctx {
    using CopyPool = pgh_detail::CopyPool;
    pgh_group* grp = nullptr;  // set: a multi-GPU group (pgh_create_group); the rest is unused
    int device = 0;
    hipStream_t stream = nullptr;  // reductions
    hipStream_t copy = nullptr;    // ingest H2D and on-device synthetic fill
    hipEvent_t copy_done = nullptr;
    hipEvent_t xsync = nullptr;    // caller-stream <-> context-stream ordering
    hipStream_t aux = nullptr;     // second reduction stream: alternate ranges of a split FINAL pass
    hipEvent_t aux_ev = nullptr;
    // The last fold issued on each stream (folds may run on several caller streams at once, e.g.
    // the param ranges of the multi-GPU overlap): the copy stream waits on all before it
    // overwrites slots, and then forgets them (later copies are ordered after those waits).
    std::vector<std::pair<hipStream_t, hipEvent_t>> fold_evs;
    // Folds that read every slab row (resident / stream / secagg): an ingest into any slot waits for
    // them.  Slot folds (pgh_fold_slots*) read only their listed slots: each is numbered, a slot
    // remembers the last one that read it, and an ingest into the slot waits for that fold alone --
    // a report's DMA does not queue behind a fold of other slots (a speculative re-fold).
    std::vector<std::pair<hipStream_t, hipEvent_t>> slab_evs;
    std::vector<int64_t> slot_read_seq;                     // per slot; 0 = not read by a slot fold
    std::deque<std::pair<int64_t, hipEvent_t>> slot_ring;  // recent slot folds on c->stream, in order
    int64_t slot_seq = 0;
    std::vector<hipEvent_t> fold_ev_pool;
    // STREAM: one event per fold with the fold front after it, so overwriting a slot waits only
    // for the fold that consumed the slot's previous client (not for the latest fold).
    struct FoldMark { hipEvent_t ev; int64_t upto; };
    std::deque<FoldMark> marks;
    std::vector<hipEvent_t> mark_pool;

    std::vector<int64_t> numel;
    int64_t P = 0, lo = 0, hi = 0, pg = 0;
    int64_t pvec = 0;  // length of the [P_shard] device vectors: pg rounded up to 64
    bool layout = false;
    // slab geometry (pgh_reserve): bw columns per block, nb blocks, bstride elements per block
    int64_t bw = 0, nb = 0, bstride = 0;
    int bshift = 62;
    int64_t bmask = 0;
    size_t block_bytes = 256u << 10;  // PGH_BLOCK_BYTES; 0 = one block (plain row-major rows)
    int synth_kind = 0;        // pgh_set_synth_kind: generator of synthetic diffs (0 Irwin-Hall, 1 fast)

    int slots = 0, dtype = PGH_F32, parties = 1;
    void* d_slab = nullptr;
    size_t slab_bytes = 0;
    float* d_ckpt = nullptr;
    float* d_out = nullptr;
    // d_ckpt holds a checkpoint (uploaded, or the output of a resident fold); a fresh slab's is
    // uninitialised memory, which a resident fold / download / patch must refuse to read
    bool ckpt_valid = false;
    float* d_acc = nullptr;
    uint64_t* d_uacc = nullptr;
    int64_t* d_sum = nullptr;
    float* d_dec = nullptr;
    float* d_w = nullptr;
    size_t w_cap = 0;
    // iterative plan: rec[k] = 1 / (double)(float)(k + 1), grown on demand, kept for the context's
    // life (a superseded table may still be read by an in-flight fold: freed at destroy)
    double* d_rec = nullptr;
    int64_t rec_cap = 0;
    std::vector<double*> rec_old;

    uint8_t* h_pin[2] = {nullptr, nullptr};
    size_t pin_slot = 0;
    hipEvent_t pin_ev[2] = {nullptr, nullptr};
    bool pin_used[2] = {false, false};
    int pin_next = 0;
    std::vector<hipEvent_t> d2h_ev;  // one per ring cell of a staged D2H (stage_d2h_pieces)
    // A staged D2H through the pinned ring: pieces of `piece` bytes of [src, src + total) into the
    // cells of the free pinned slots, each followed by d2h_ev[cell].  piped: src is a fold's result
    // with range marks; each piece is issued (on the copy stream) once the host sees every mark
    // covering it complete -- no cross-stream wait on the device, which sent the pieces to blit
    // kernels that slowed the ranges beside them (profiles/r05k/-r05m/, r05aa/).
    struct D2HRing {
        const uint8_t* src = nullptr;
        size_t total = 0, piece = 0, per_slot = 0, cells = 0, n_pieces = 0, queued = 0, done = 0;
        int free_slot[2] = {0, 1};
        int n_free = 0;
        hipStream_t s = nullptr;
        bool piped = false;
        uint8_t* base = nullptr;  // the cells of a piped ring: h_d2h (own_d2h), else the free pinned slots
    };
    // The new checkpoint's D2H as the FINAL pass of a report-time close starts it: the pieces whose
    // ranges finished while the later ranges were still being issued (pgh_slots.cpp); the patch /
    // download that follows adopts the ring.  Dropped with the marks (clear_final_marks) or when a
    // staging copy takes a pinned slot (take_pin_slot).
    D2HRing pre_d2h;
    bool pre_d2h_valid = false;
    // A piped ring's pieces on a stream and in page-locked cells of their own (PGH_D2H_STREAM,
    // default 1): on the copy stream they queued behind the last reports' H2D, and they waited for
    // a staging slot those reports still held -- with reports back to back, until every report had
    // landed.  The stream is primed with a small H2D when made, so the runtime sends its D2H to an
    // SDMA engine (r05ae).  (Rounds 6's K6 k_copy_to_host, pieces copied out by a kernel beside an H2D
    // backlog, was removed: copying a piece right behind the FINAL ranges that wrote it on another
    // stream, it read ranges that had not run yet -- profiles/r06s/.)
    bool own_d2h = true;
    int d2h_mode = 1;
    hipStream_t d2h = nullptr;
    uint8_t* h_d2h = nullptr;
    size_t d2h_cap = 0;
    int copy_threads = 8;
    std::vector<int> local_cpus;  // PGH_NUMA (default on): the GPU's socket, for the copy pool + pinned ring
    std::unique_ptr<CopyPool> pool_copy;

    // secagg shares as State bytes: varint payloads in HBM + their chunk table (k_varint_decode)
    // Each decode runs on its own stream (dec) behind its message's DMAs, so the copy stream's next
    // DMA does not queue behind it; the HBM bytes and chunk table alternate between two buffers (the
    // DMA of one message beside the decode of the one before).
    struct VarintBuf {
        uint8_t* bytes = nullptr;
        size_t cap = 0;
        pgh::VChunk* tab = nullptr;
        size_t tab_cap = 0;
        hipEvent_t done = nullptr;  // the last decode that read this buffer
        bool used = false;
    };
    VarintBuf vbuf[2];
    int vbuf_next = 0;
    hipStream_t dec = nullptr;
    hipEvent_t dec_in = nullptr;     // copy stream -> dec: a message's bytes and table have landed
    hipEvent_t dec_last = nullptr;   // the last decode issued: folds wait for it (order_after_ingest)
    pgh::VChunk* h_vtab = nullptr;   // pinned host image of a chunk table
    size_t vtab_cap = 0;
    hipEvent_t vtab_ev = nullptr;    // the last table upload (h_vtab reusable after it)
    bool vtab_used = false;
    // page-locked fp32 State messages (below) stage through this buffer
    uint8_t* d_vbytes = nullptr;
    size_t vbytes_cap = 0;
    // page-locked fp32 State messages (pgh_ingest_state): DMA'd whole into d_vbytes, gathered into the
    // slab row by k_gather_f32 with this chunk table (PGH_PINNED_GATHER=0: one DMA per payload piece)
    pgh::GChunk* d_gtab = nullptr;
    pgh::GChunk* h_gtab = nullptr;  // pinned
    size_t gtab_cap = 0;
    hipEvent_t gtab_ev = nullptr;    // the last table upload (h_gtab reusable after it)
    hipEvent_t gdma_ev = nullptr;    // the last message DMA (the caller's buffer is free after it)
    bool gtab_used = false;
    bool pinned_gather = true;
    // Ranged report ingest (pgh_set_ingest_ranges): a State diff goes to HBM in chunks of
    // INGEST_CHUNK params, each followed by rng_ev[k] on the copy stream, so that the FINAL pass of
    // a report-time close that starts while the last report's DMA is still in flight folds each
    // param range as soon as its bytes have landed.  copy_seq counts the data operations issued on
    // the copy stream; the ranged close applies only while rng_seq == copy_seq (nothing issued on
    // the copy stream since the latest ranged ingest) and rng_n chunks cover the shard.
    bool ingest_ranges = false;
    std::vector<hipEvent_t> rng_ev;
    uint64_t copy_seq = 0, rng_seq = ~0ull;
    int rng_n = 0;
    bool warmup_skipped = false;  // pgh_create's warm-up failed (e.g. no device memory left): skipped
    int64_t vec_min = 0;      // [P_shard] device vectors at least this long (group collectives)
    // Pipelined close: a resident fold's FINAL pass runs as final_split param ranges, each followed by
    // an event; a D2H of the new checkpoint (patch / download) then runs on the copy stream, piece by
    // piece behind the range that wrote it, so the HBM -> host copy overlaps the rest of the fold
    // (PGH_FINAL_RANGES, shards of >= 1 M params; opt-in, see final_split below).
    struct RangeMark { int64_t end; hipEvent_t ev; };
    std::vector<RangeMark> final_marks;
    std::vector<hipEvent_t> rmark_pool;
    // PGH_FINAL_RANGES (opt-in): split the FINAL pass of resident folds into this many param ranges
    // with marks, so a following D2H starts behind the first range.  Off by default: each extra
    // launch costs its drain (ResNet-18 fold 7.45 ms as 4 ranges on two streams vs 6.91 ms as one,
    // r02r), about what the earlier D2H start saves in a close (report closes within noise, r02l/r02r).
    int final_split = 1;
    int64_t client_base = 0;  // synthetic client k is generated as global client client_base + k

    std::vector<int64_t> slot_client;  // client held by each slot and not yet folded, or -1
    std::vector<float> weights;
    bool weights_on_device = false;

    bool streaming = false;
    int slot_mode = -1;  // pgh_fold_slots: averaging mode of the cycle being folded slot by slot
    int kind = 0;
    int fold_batch = 1;
    int64_t folded = 0;  // stream: clients [0, folded) are in the running state

    int variant = PGH_DEFAULT_VARIANT;
    struct Timed { hipEvent_t a, b; uint64_t bytes; };
    std::vector<Timed> pending;
    std::vector<hipEvent_t> pool;
    pgh_stats_t st{};
    std::string err;
};

#define CK(c, expr)                                                                            \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((c), PGH_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                                   \
    } while (0)

#define RC(expr)            \
    do {                    \
        int r_ = (expr);    \
        if (r_) return r_;  \
    } while (0)

namespace pgh_detail {

// ---- errors, device selection, time ------------------------------------------------------------
// Set the context's (or, with c == NULL, the calling thread's creation) error message; returns code.
int fail(pgh_ctx* c, int code, const char* fmt, ...);
int vfail(pgh_ctx* c, int code, const char* fmt, va_list ap);

struct DeviceGuard {  // select the context's GPU for the call, restore the caller's after
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

double now_ms();

// ---- state checks and slab geometry -------------------------------------------------------------
inline size_t esize(int dtype) { return dtype == PGH_F32 ? 4 : 8; }
inline bool valid_mode(int m) { return m == PGH_MEAN || m == PGH_ITERATIVE_MEAN || m == PGH_WEIGHTED_MEAN; }
int check_ready(pgh_ctx* c);
int check_dtype(pgh_ctx* c, int dtype);
int check_ckpt(pgh_ctx* c, const char* what);
void free_slab(pgh_ctx* c);

// Slab geometry for kernels (off = 0) and the start of a slot's first row inside block 0.
inline pgh::SlabMap slab_map(const pgh_ctx* c) { return pgh::SlabMap{c->bw, c->bstride, c->bshift, c->bmask, 0}; }
inline uint8_t* slot_row(pgh_ctx* c, int slot, int party) {
    const size_t row = (size_t)slot * c->parties + party;
    return (uint8_t*)c->d_slab + row * (size_t)c->bw * esize(c->dtype);
}

// Where host bytes land: a slab row (blocked) or a [p] vector (one block).
struct Dest {
    uint8_t* base;       // row start in block 0 / vector start
    pgh::SlabMap map;
    size_t es;
    int64_t len = 0;     // a slab row: its elements (the last block's columns past it are padding)
};
inline Dest row_dest(pgh_ctx* c, int slot, int party) {
    return Dest{slot_row(c, slot, party), slab_map(c), esize(c->dtype), c->pg};
}
inline Dest vec_dest(void* v, int64_t n, size_t es) { return Dest{(uint8_t*)v, pgh::single_block(n), es}; }

// ---- kernel timing -------------------------------------------------------------------------------
hipEvent_t take_event(pgh_ctx* c);
int collect_timings(pgh_ctx* c);

// Bracket a launch with an event pair on `s`.
template <class F>
int timed_launch(pgh_ctx* c, hipStream_t s, uint64_t bytes, F&& launch) {
    if (c->pending.size() >= 4096) RC(collect_timings(c));
    hipEvent_t a = take_event(c), b = take_event(c);
    if (!a || !b) return fail(c, PGH_E_HIP, "hipEventCreate failed");
    CK(c, hipEventRecord(a, s));
    hipError_t e = launch();
    if (e != hipSuccess) {
        c->pool.push_back(a); c->pool.push_back(b);
        return fail(c, PGH_E_HIP, "kernel launch failed: %s", hipGetErrorString(e));
    }
    CK(c, hipEventRecord(b, s));
    c->pending.push_back({a, b, bytes});
    return PGH_OK;
}

// ---- host <-> HBM --------------------------------------------------------------------------------
struct Piece {
    const uint8_t* src;
    size_t n;
};
struct OutPiece {
    uint8_t* dst;
    size_t n;
};

// HBM -> host results move in pieces of at most D2H_PIECE, the later pieces' DMAs beside the host
// copy-out of the earlier ones (r01ac: 4, 8, 16 MiB within the noise of the 47 MB report-time close;
// with the parallel pre-fault, r01ak, 8 MiB pieces closed in 2.3-2.4 ms vs 2.6-2.7 for one piece).
constexpr size_t D2H_PIECE = 8u << 20;
constexpr size_t D2H_OWN_CELLS = 8;  // a piped ring's own cells: 64 MiB at most (ResNet-18: 6 pieces)
// Ranged report ingest (pgh_set_ingest_ranges): one chunk = the params of one D2H piece = two
// 4 MiB FINAL ranges of a report-time close (pgh_slots.cpp).
constexpr int64_t INGEST_CHUNK = (int64_t)(D2H_PIECE / 4);

bool is_pinned(const void* p);
// src_room: bytes readable at src past the n elements (a staging slot's unused rest); a range that
// ends a slab row whose last block is partial then goes as full blocks in one 2D copy (the padding
// columns take whatever follows in the slot) instead of a 2D copy plus a tail copy.
int h2d_range(pgh_ctx* c, const Dest& d, int64_t i0, const uint8_t* src, int64_t n, hipStream_t s,
              size_t src_room = 0);
int stage_pieces_h2d(pgh_ctx* c, const Dest& dst, const std::vector<Piece>& pieces);
int stage_pieces_h2d_ranged(pgh_ctx* c, const Dest& dst, const std::vector<Piece>& pieces, size_t total);
bool ranged_ingest_valid(const pgh_ctx* c);
int stage_h2d(pgh_ctx* c, const Dest& dst, const uint8_t* src, size_t n, bool pinned_src);
void scatter_out(const uint8_t* src, size_t off, size_t len, const std::vector<OutPiece>& pieces, CopyPool& pool);
void prefault_small_any(uint8_t* p, size_t n);
void prefault_parallel(uint8_t* p, size_t n, CopyPool& pool);
int stage_d2h_pieces(pgh_ctx* c, const uint8_t* src, const std::vector<OutPiece>& pieces, hipStream_t s,
                     const std::function<void()>& overlap = nullptr, bool marks = false);
// may_wait = false: both pinned slots still busy -> r->n_free == 0 (nothing set up) instead of waiting
int d2h_ring_begin(pgh_ctx* c, pgh_ctx::D2HRing* r, const uint8_t* src, size_t total, hipStream_t s, bool piped,
                   bool may_wait = true);
int d2h_issue_ready(pgh_ctx* c, pgh_ctx::D2HRing* r);  // piped: every piece whose marks have fired, no wait
int take_pin_slot(pgh_ctx* c, int* slot);  // the next pinned staging slot, free of earlier DMAs
int state_shard_spans(pgh_ctx* c, const uint8_t* pb, size_t n, std::vector<std::pair<size_t, size_t>>* out,
                      const char* what);
// page-locked blocks marked async (pgh_host_async): DMAs from them are recorded, not waited for
bool host_async(const void* p, size_t n);
int host_dma_queued(pgh_ctx* c, const void* p, size_t n, hipStream_t s);

// ---- ordering between ingest copies and folds -----------------------------------------------------
int order_after_ingest(pgh_ctx* c, hipStream_t s);
void release_slot_fold_events(pgh_ctx* c);
int record_slab_fold(pgh_ctx* c, hipStream_t s);
int record_slot_fold(pgh_ctx* c, const int32_t* slots, int n);
int order_slot_overwrite(pgh_ctx* c, int slot);
int order_before_overwrite(pgh_ctx* c);
int record_fold(pgh_ctx* c, hipStream_t s);
void clear_marks(pgh_ctx* c);
int order_stream_overwrite(pgh_ctx* c, int64_t last_client);
int record_mark(pgh_ctx* c, hipStream_t s, int64_t upto);
int join_in(pgh_ctx* c, hipStream_t cs);
int join_out(pgh_ctx* c, hipStream_t cs);

// ---- pipelined close: range marks of the last resident fold -----------------------------------------
void clear_final_marks(pgh_ctx* c);
int add_final_mark(pgh_ctx* c, hipStream_t s, int64_t end);
hipStream_t range_stream(const pgh_ctx* c, hipStream_t s, int k);
int fork_aux(pgh_ctx* c, hipStream_t s);
int join_aux(pgh_ctx* c, hipStream_t s);
int final_ranges(const pgh_ctx* c);
int64_t range_edge(const pgh_ctx* c, int k, int K);

// ---- folds ---------------------------------------------------------------------------------------
int sync_weights(pgh_ctx* c, hipStream_t s);
int ensure_recips(pgh_ctx* c, int64_t n, hipStream_t s);
int fixed_point_divisor(pgh_ctx* c, int base, int prec, float* div);
int fedavg_divisor(pgh_ctx* c, int mode, int64_t n, float* div);

// What a FINAL fold pass writes (fedavg: ckpt - avg; secagg: sum/dec) and over which param range.
struct FinalArgs {
    const float* ckpt = nullptr;  // shard base pointers; the launch touches [off, off + len)
    float* out = nullptr;
    int64_t* sum = nullptr;
    float* dec = nullptr;
    float divisor = 1.f;
    int64_t off = 0;   // param range within the shard
    int64_t len = -1;  // -1 = to the end of the shard
};
int fold_run(pgh_ctx* c, int kind, int64_t c0, int64_t n, bool final, const FinalArgs& fa, hipStream_t s);
int64_t ready_run(pgh_ctx* c, int64_t from);
int check_no_gaps(pgh_ctx* c, int64_t from, int64_t run);
int maybe_fold(pgh_ctx* c, bool force);
int claim_slot(pgh_ctx* c, int64_t client, int* slot_out);
int mark_ingested(pgh_ctx* c, int64_t client, int slot);
int resident_count(pgh_ctx* c, int64_t* n_out);

}  // namespace pgh_detail
