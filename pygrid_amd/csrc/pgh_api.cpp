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
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pgh_api.h"
#include "pgh_internal.h"
#include "pgh_kernels.h"
#include "pgh_state.h"

namespace {
constexpr int KIND_SECAGG = 3;  // stream kind besides the three fedavg modes
}

// Host copy engine: a persistent pool that splits one batch of (dst, src, n) segments evenly
// by bytes across its threads (the caller's thread takes the first share).  Used to fill and
// drain the pinned staging slots, where payload pieces are many and mostly small.
// memcpy with non-temporal 16-byte stores for big copies into staging / output buffers (no
// read-for-ownership of the destination, which is written once and then read by the DMA engine or
// handed to the caller; r01ab).
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

// Bind the calling thread to `cpus` (no-op when empty or refused).
void bind_thread(const std::vector<int>& cpus) {
    if (cpus.empty()) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
}

// CPUs on the GPU's own socket (its PCI device's local_cpulist) that this process may run on; empty
// when unknown.  Staging copies and pinned buffers there keep the host side of every H2D / D2H off
// the socket interconnect (a 2-socket node: GPUs 0-3 on one socket, 4-7 on the other).
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

struct pgh_ctx {
    pgh_group* grp = nullptr;  // set: a multi-GPU group (pgh_create_group); the rest is unused
    int device = 0;
    hipStream_t stream = nullptr;  // reductions
    hipStream_t copy = nullptr;    // ingest H2D and on-device synthetic fill
    hipEvent_t copy_done = nullptr;
    hipEvent_t xsync = nullptr;    // caller-stream <-> context-stream ordering
    hipStream_t aux = nullptr;     // second reduction stream: alternate ranges of a split FINAL pass
    hipEvent_t aux_ev = nullptr;
    // Speculative close (pgh_fold_peek): the FINAL pass of the fold state as it stands, written to
    // d_out and copied to the pinned h_peek on peek_stream (D2H beside the ingest H2D), valid while
    // state_gen is unchanged -- every fold, rewind, restart, weight or checkpoint change bumps it.
    hipStream_t peek_stream = nullptr;
    hipEvent_t peek_ev = nullptr;
    // the D2H runs in D2H_PIECE pieces, an event behind each: the peek thread copies a piece out as
    // soon as it lands (the copy-out overlaps the rest of the D2H instead of following all of it)
    std::vector<hipEvent_t> peek_piece_ev;
    size_t peek_pieces = 0;    // pieces of the last peek's D2H
    float* h_peek = nullptr;   // pinned, peek_cap floats
    size_t peek_cap = 0;
    float* d_peek = nullptr;   // [pvec]: the peeked new checkpoint (swapped with d_ckpt on commit)
    // pgh_fold_peek_into: a host thread waits for the peek's D2H and copies its payload slices into
    // the caller's framed output while the cycle is still open (the close then only commits)
    std::thread pk_thread;
    std::mutex pk_mu;
    std::condition_variable pk_cv;
    bool pk_stop = false, pk_busy = false;
    uint64_t pk_gen = 0;       // peek the posted job copies
    uint64_t pk_done_gen = 0;  // peek whose payloads are in pk_done_out
    uint8_t* pk_out = nullptr;
    const uint8_t* pk_done_out = nullptr;
    std::vector<std::pair<uint8_t*, size_t>> pk_pieces;
    std::unique_ptr<CopyPool> pool_peek;
    uint64_t state_gen = 1;
    uint64_t peek_gen = 0;  // state_gen the peek was taken at (0: none)
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
    int copy_threads = 8;
    std::vector<int> local_cpus;  // PGH_NUMA (default on): the GPU's socket, for the copy pool + pinned ring
    std::unique_ptr<CopyPool> pool_copy;

    // secagg shares as State bytes: varint payloads in HBM + their chunk table (k_varint_decode)
    uint8_t* d_vbytes = nullptr;
    size_t vbytes_cap = 0;
    pgh::VChunk* d_vtab = nullptr;
    pgh::VChunk* h_vtab = nullptr;  // pinned
    size_t vtab_cap = 0;
    hipEvent_t vtab_ev = nullptr;
    bool vtab_used = false;
    // page-locked fp32 State messages (pgh_ingest_state): DMA'd whole into d_vbytes, gathered into the
    // slab row by k_gather_f32 with this chunk table (PGH_PINNED_GATHER=0: one DMA per payload piece)
    pgh::GChunk* d_gtab = nullptr;
    pgh::GChunk* h_gtab = nullptr;  // pinned
    size_t gtab_cap = 0;
    hipEvent_t gtab_ev = nullptr;    // the last table upload (h_gtab reusable after it)
    hipEvent_t gdma_ev = nullptr;    // the last message DMA (the caller's buffer is free after it)
    bool gtab_used = false;
    bool pinned_gather = true;
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
    // Saved slot-fold states (pgh_fold_mark / pgh_fold_rewind: speculative report-time folds).  A mark
    // takes over the d_acc buffer it names (d_acc moves on to a spare one), so neither saving nor
    // rewinding copies: after a rewind the next slot fold reads its running state from the mark's
    // buffer (acc_src) and writes d_acc.
    struct SavedFold { float* buf; int64_t folded; int mode; };
    std::map<int, SavedFold> fold_marks;
    std::vector<float*> acc_spare;     // [pvec] fold-state buffers not in use
    const float* acc_src = nullptr;    // set by a rewind: the running state lives here, not in d_acc
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

namespace {

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

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

size_t esize(int dtype) { return dtype == PGH_F32 ? 4 : 8; }

void release_slot_fold_events(pgh_ctx* c);
void peek_job_wait(pgh_ctx* c);
void peek_thread_stop(pgh_ctx* c);

void free_slab(pgh_ctx* c) {
    peek_job_wait(c);  // the peek thread reads h_peek
    if (c->peek_stream) (void)hipStreamSynchronize(c->peek_stream);  // a peek's D2H reads d_peek
    (void)hipFree(c->d_peek); c->d_peek = nullptr;
    if (c->h_peek) (void)hipHostFree(c->h_peek);
    c->h_peek = nullptr; c->peek_cap = 0; c->peek_gen = 0;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    for (auto& fe : c->fold_evs) (void)hipEventSynchronize(fe.second);  // folds on caller streams
    (void)hipFree(c->d_slab); c->d_slab = nullptr; c->slab_bytes = 0;
    (void)hipFree(c->d_ckpt); c->d_ckpt = nullptr;
    (void)hipFree(c->d_out); c->d_out = nullptr;
    c->ckpt_valid = false; ++c->state_gen;
    for (auto& m : c->final_marks) c->rmark_pool.push_back(m.ev);
    c->final_marks.clear();
    (void)hipFree(c->d_acc); c->d_acc = nullptr;
    for (auto& m : c->fold_marks) (void)hipFree(m.second.buf);
    c->fold_marks.clear();
    for (float* b : c->acc_spare) (void)hipFree(b);
    c->acc_spare.clear();
    c->acc_src = nullptr;
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

// Slab geometry for kernels (off = 0) and the start of a slot's first row inside block 0.
pgh::SlabMap slab_map(const pgh_ctx* c) { return pgh::SlabMap{c->bw, c->bstride, c->bshift, c->bmask, 0}; }

uint8_t* slot_row(pgh_ctx* c, int slot, int party) {
    const size_t row = (size_t)slot * c->parties + party;
    return (uint8_t*)c->d_slab + row * (size_t)c->bw * esize(c->dtype);
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

// Where host bytes land: a slab row (blocked) or a [p] vector (one block).
struct Dest {
    uint8_t* base;       // row start in block 0 / vector start
    pgh::SlabMap map;
    size_t es;
};
Dest row_dest(pgh_ctx* c, int slot, int party) { return Dest{slot_row(c, slot, party), slab_map(c), esize(c->dtype)}; }
Dest vec_dest(void* v, int64_t n, size_t es) { return Dest{(uint8_t*)v, pgh::single_block(n), es}; }

// Elements [i0, i0 + n) of one row from contiguous host memory: the partial first block, the
// whole blocks as ONE 2-D copy (block rows bstride apart), the partial last block.
int h2d_range(pgh_ctx* c, const Dest& d, int64_t i0, const uint8_t* src, int64_t n, hipStream_t s) {
    const size_t es = d.es;
    if (n <= 0) return PGH_OK;
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
    const int64_t full = (i1 - i) / bw;
    if (full > 0) {
        CK(c, hipMemcpy2DAsync(d.base + (size_t)d.map.at(i) * es, (size_t)d.map.bstride * es, src, (size_t)bw * es,
                               (size_t)bw * es, (size_t)full, hipMemcpyHostToDevice, s));
        src += (size_t)(full * bw) * es;
        i += full * bw;
    }
    if (i < i1)  // tail
        CK(c, hipMemcpyAsync(d.base + (size_t)d.map.at(i) * es, src, (size_t)(i1 - i) * es, hipMemcpyHostToDevice, s));
    return PGH_OK;
}

hipEvent_t take_event(pgh_ctx* c) {
    if (!c->pool.empty()) { hipEvent_t e = c->pool.back(); c->pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
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

bool is_pinned(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    return attr.type == hipMemoryTypeHost;
}

struct Piece {
    const uint8_t* src;
    size_t n;
};

// Concatenated host pieces -> HBM at `dst`, through the pinned ring: each slot is filled by
// (multi-threaded) host copies of as many pieces as fit, then DMA'd while the next slot fills.
int stage_pieces_h2d(pgh_ctx* c, const Dest& dst, const std::vector<Piece>& pieces) {
    const double t0 = now_ms();
    size_t total = 0, done = 0, pi = 0, poff = 0;
    for (auto& p : pieces) total += p.n;
    while (done < total) {
        const int slot = c->pin_next;
        c->pin_next ^= 1;
        if (c->pin_used[slot]) CK(c, hipEventSynchronize(c->pin_ev[slot]));
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
        RC(h2d_range(c, dst, (int64_t)(done / dst.es), c->h_pin[slot], (int64_t)(fill / dst.es), c->copy));
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

struct OutPiece {
    uint8_t* dst;
    size_t n;
};

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
// instead of taking a page fault per 4 KiB (PGH_PREFAULT=0 turns it off).
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

// HBM -> host results move in pieces of at most D2H_PIECE, the DMA of piece i + 1 beside the host
// copy-out of piece i (r01ac: 4, 8, 16 MiB within the noise of the 47 MB report-time close; with the
// parallel pre-fault, r01ak, 8 MiB pieces closed in 2.3-2.4 ms vs 2.6-2.7 for one piece).
constexpr size_t D2H_PIECE = 8u << 20;

// HBM bytes at `src` (after the work already on stream `s`) -> host pieces, through the pinned
// ring: the DMA of one slot overlaps the host copy-out of the previous one.  `overlap`, if given,
// is host work run while the first DMA is in flight (the checkpoint template's framing copy).
// marks: src is the resident checkpoint: when its last fold left range marks, the DMAs run on the
// copy stream, each behind the range that wrote its bytes (the rest of the fold continues).
int stage_d2h_pieces(pgh_ctx* c, const uint8_t* src, const std::vector<OutPiece>& pieces, hipStream_t s,
                     const std::function<void()>& overlap = nullptr, bool marks = false) {
    size_t total = 0;
    for (auto& p : pieces) total += p.n;
    const bool piped = marks && !c->final_marks.empty();
    if (piped) s = c->copy;
    size_t off = 0;
    int prev_slot = -1;
    size_t prev_off = 0, prev_len = 0;
    while (off < total || prev_slot >= 0) {
        int cur_slot = -1;
        size_t cur_len = 0;
        if (off < total) {
            cur_slot = c->pin_next;
            c->pin_next ^= 1;
            if (c->pin_used[cur_slot]) CK(c, hipEventSynchronize(c->pin_ev[cur_slot]));
            cur_len = std::min({total - off, c->pin_slot, D2H_PIECE});
            if (piped) {  // wait for EVERY fold range the piece's floats come from: the ranges
                          // alternate over two streams, so the last one's mark orders nothing else
                const int64_t first = (int64_t)(off / 4), last = (int64_t)((off + cur_len + 3) / 4);
                int64_t start = 0;
                for (auto& m : c->final_marks) {
                    if (start >= last) break;
                    if (m.end > first) CK(c, hipStreamWaitEvent(s, m.ev, 0));
                    start = m.end;
                }
            }
            CK(c, hipMemcpyAsync(c->h_pin[cur_slot], src + off, cur_len, hipMemcpyDeviceToHost, s));
            CK(c, hipEventRecord(c->pin_ev[cur_slot], s));
            c->pin_used[cur_slot] = true;
        }
        if (overlap && off == 0) overlap();
        if (prev_slot >= 0) {
            CK(c, hipEventSynchronize(c->pin_ev[prev_slot]));
            scatter_out(c->h_pin[prev_slot], prev_off, prev_len, pieces, *c->pool_copy);
        }
        prev_slot = cur_slot;
        prev_off = off;
        prev_len = cur_len;
        off += cur_len;
    }
    return PGH_OK;
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

// Stream `s` waits for every ingest copy / synthetic fill issued so far.
int order_after_ingest(pgh_ctx* c, hipStream_t s) {
    CK(c, hipEventRecord(c->copy_done, c->copy));
    CK(c, hipStreamWaitEvent(s, c->copy_done, 0));
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

// Forget every saved slot-fold state (and a pending rewind: the caller discards the fold state too).
// Their buffers become spares; anything still reading them is ordered on c->stream before the next
// writer (a slot fold on the same stream).
void drop_fold_marks(pgh_ctx* c) {
    for (auto& m : c->fold_marks)
        if (m.second.buf) c->acc_spare.push_back(m.second.buf);
    c->fold_marks.clear();
    c->acc_src = nullptr;
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
struct FinalArgs {
    const float* ckpt = nullptr;  // shard base pointers; the launch touches [off, off + len)
    float* out = nullptr;
    int64_t* sum = nullptr;
    float* dec = nullptr;
    float divisor = 1.f;
    int64_t off = 0;   // param range within the shard
    int64_t len = -1;  // -1 = to the end of the shard
};

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
    ++c->state_gen;
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

bool valid_mode(int m) { return m == PGH_MEAN || m == PGH_ITERATIVE_MEAN || m == PGH_WEIGHTED_MEAN; }

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

}  // namespace

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

// ---- page-locked blocks whose DMAs may outlive the ingest call -------------------------------------
// pgh_host_async marks a pgh_host_alloc block: an ingest from it then returns once the DMA is queued
// (not done), and records the DMA's event here; pgh_host_wait(p, n) waits for every DMA still reading
// [p, p + n) (any context, any GPU) before the owner reuses or frees the block.  Unmarked page-locked
// memory keeps the synchronous contract (the call waits for its copies).
namespace {
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
}  // namespace

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
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&c->copy_done, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->xsync, hipEventDisableTiming) == hipSuccess &&
              hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&c->aux_ev, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->pin_ev[0], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->pin_ev[1], hipEventDisableTiming) == hipSuccess;
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
    peek_thread_stop(c);
    for (auto& t : c->pending) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    clear_marks(c);
    for (auto e : c->mark_pool) (void)hipEventDestroy(e);
    (void)hipFree(c->d_rec);
    for (double* p : c->rec_old) (void)hipFree(p);
    (void)hipFree(c->d_vbytes);
    (void)hipFree(c->d_vtab);
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
    for (hipEvent_t e : {c->copy_done, c->xsync, c->aux_ev})
        if (e) (void)hipEventDestroy(e);
    for (auto e : c->fold_ev_pool) (void)hipEventDestroy(e);
    for (auto e : c->rmark_pool) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    if (c->peek_ev) (void)hipEventDestroy(c->peek_ev);
    for (auto e : c->peek_piece_ev) (void)hipEventDestroy(e);
    if (c->peek_stream) (void)hipStreamDestroy(c->peek_stream);
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
    drop_fold_marks(c);
    release_slot_fold_events(c);  // c->stream is idle (synchronised above)
    peek_job_wait(c);             // the caller may drop the output a peek is copying into after this
    ++c->state_gen;
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
int pinned_gather_ingest(pgh_ctx* c, const uint8_t* pb, const std::vector<Piece>& pieces, int slot);
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
    if (n && !pieces.empty() && c->pinned_gather && is_pinned(pb)) {
        // Page-locked message (a report decoded straight into pgh_host_alloc memory,
        // pygrid_amd.report.PinnedPool): no staging copy.  The part of the message holding this
        // shard's payloads goes to HBM in ONE DMA (a few hundred bytes of framing ride along) and
        // k_gather_f32 moves the payloads into the slab row; the call waits for the DMA only (the
        // buffer is borrowed), the gather runs on behind it on the copy stream.
        const double t0 = now_ms();
        RC(pinned_gather_ingest(c, pb, pieces, slot));
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
// -> its region of the HBM byte buffer, on the copy stream.  Nothing is decoded yet.
int stage_share_msg(pgh_ctx* c, ShareMsg& m) {
    const double t0 = now_ms();
    const size_t nk = m.chunks.size();
    size_t k = 0;
    while (k < nk) {
        const int ps = c->pin_next;
        c->pin_next ^= 1;
        if (c->pin_used[ps]) CK(c, hipEventSynchronize(c->pin_ev[ps]));
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
        CK(c, hipMemcpyAsync(c->d_vbytes + s0, pin, fill, hipMemcpyHostToDevice, c->copy));
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
// DMA to d_vbytes, the gather table behind it, then k_gather_f32 into the slot's row.
int pinned_gather_ingest(pgh_ctx* c, const uint8_t* pb, const std::vector<Piece>& pieces, int slot) {
    const size_t a = (size_t)(pieces.front().src - pb) & ~(size_t)63;
    const size_t b = (size_t)(pieces.back().src - pb) + pieces.back().n;
    std::vector<pgh::GChunk> tab;
    int64_t dst = 0;
    size_t total = 0;
    for (auto& p : pieces) {
        const int64_t nf = (int64_t)(p.n / 4);
        const int64_t src = (int64_t)((size_t)(p.src - pb) - a);
        for (int64_t k = 0; k < nf; k += pgh::GATHER_CHUNK)
            tab.push_back({src + 4 * k, dst + k, (int32_t)std::min<int64_t>(pgh::GATHER_CHUNK, nf - k), 0});
        dst += nf;
        total += p.n;
    }
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
    CK(c, hipMemcpyAsync(c->d_gtab, c->h_gtab, tb, hipMemcpyHostToDevice, c->copy));
    CK(c, hipEventRecord(c->gtab_ev, c->copy));
    c->gtab_used = true;
    CK(c, hipMemcpyAsync(c->d_vbytes, pb + a, b - a, hipMemcpyHostToDevice, c->copy));
    const bool async = host_async(pb + a, b - a);
    if (async) RC(host_dma_queued(c, pb + a, b - a, c->copy));  // the block's owner waits (pgh_host_wait)
    else CK(c, hipEventRecord(c->gdma_ev, c->copy));
    const Dest d = row_dest(c, slot, 0);
    const hipError_t e = pgh::launch_gather_f32(c->d_vbytes, c->d_gtab, (int)tab.size(), (float*)d.base, d.map,
                                                c->copy);
    if (e != hipSuccess) return fail(c, PGH_E_HIP, "gather launch failed: %s", hipGetErrorString(e));
    if (!async) CK(c, hipEventSynchronize(c->gdma_ev));
    c->st.h2d_bytes_total += total;
    return PGH_OK;
}

// Every party validated: one chunk table for all of them, then one decode per party into its
// slab row (the shard's range), on the copy stream.
int decode_share_msgs(pgh_ctx* c, std::vector<ShareMsg>& msgs, int slot) {
    size_t nk = 0;
    for (auto& m : msgs) nk += m.chunks.size();
    if (nk == 0) return PGH_OK;  // every tensor empty
    const size_t tb = nk * sizeof(pgh::VChunk);
    if (!c->vtab_ev) CK(c, hipEventCreateWithFlags(&c->vtab_ev, hipEventDisableTiming));
    if (c->vtab_used) CK(c, hipEventSynchronize(c->vtab_ev));  // the previous table upload read h_vtab
    if (tb > c->vtab_cap) {
        if (c->h_vtab) (void)hipHostFree(c->h_vtab);
        c->h_vtab = nullptr;
        size_t cap = 0;
        void* d = c->d_vtab;
        RC(grow_device(c, &d, &cap, tb, "varint chunk table"));
        c->d_vtab = (pgh::VChunk*)d;
        if (hipHostMalloc((void**)&c->h_vtab, cap, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            c->vtab_cap = 0;
            return fail(c, PGH_E_OOM, "pinned chunk table of %zu bytes failed", cap);
        }
        c->vtab_cap = cap;
        c->vtab_used = false;
    }
    size_t at = 0;
    for (auto& m : msgs) {
        std::memcpy(c->h_vtab + at, m.chunks.data(), m.chunks.size() * sizeof(pgh::VChunk));
        at += m.chunks.size();
    }
    CK(c, hipMemcpyAsync(c->d_vtab, c->h_vtab, tb, hipMemcpyHostToDevice, c->copy));
    CK(c, hipEventRecord(c->vtab_ev, c->copy));
    c->vtab_used = true;
    at = 0;
    for (size_t s = 0; s < msgs.size(); ++s) {
        const int n = (int)msgs[s].chunks.size();
        const hipError_t e = pgh::launch_varint_decode(c->d_vbytes, c->d_vtab + at, n,
                                                       (int64_t*)slot_row(c, slot, (int)s), slab_map(c), c->lo, c->hi,
                                                       c->copy);
        if (e != hipSuccess) return fail(c, PGH_E_HIP, "varint decode launch failed: %s", hipGetErrorString(e));
        at += (size_t)n;
    }
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
    DeviceGuard g(c->device);
    int slot = 0;
    RC(claim_slot(c, client, &slot));
    RC(grow_device(c, (void**)&c->d_vbytes, &c->vbytes_cap, total + 16, "share payload buffer"));
    for (auto& m : msgs) RC(stage_share_msg(c, m));
    for (int s = 0; s < n_parties; ++s) RC(check_share_msg(c, &msgs[(size_t)s], client, s));
    RC(decode_share_msgs(c, msgs, slot));
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
    c->ckpt_valid = false; ++c->state_gen;  // the resident checkpoint is used as scratch here
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
    ++c->state_gen;
    return PGH_OK;
}

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
    c->ckpt_valid = false; ++c->state_gen;
    clear_final_marks(c);
    RC(stage_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), (const uint8_t*)ckpt, bytes, is_pinned(ckpt)));
    c->ckpt_valid = true; ++c->state_gen;
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
    c->ckpt_valid = false; ++c->state_gen;
    clear_final_marks(c);
    RC(stage_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), src, shard, is_pinned(ckpt)));
    c->ckpt_valid = true; ++c->state_gen;
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
    c->ckpt_valid = false; ++c->state_gen;
    clear_final_marks(c);
    RC(stage_pieces_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), pieces));
    c->ckpt_valid = true; ++c->state_gen;
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
    peek_job_wait(c);  // a peek's payload copy may still be writing the same output
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
namespace {
// Wait until the peek thread is idle (its copy read h_peek and wrote the caller's buffer).
void peek_job_wait(pgh_ctx* c) {
    std::unique_lock<std::mutex> lk(c->pk_mu);
    c->pk_cv.wait(lk, [c] { return !c->pk_busy; });
}

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

void peek_thread_stop(pgh_ctx* c) {
    if (!c->pk_thread.joinable()) return;
    {
        std::lock_guard<std::mutex> lk(c->pk_mu);
        c->pk_stop = true;
    }
    c->pk_cv.notify_all();
    c->pk_thread.join();
}
}  // namespace

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
    c->ckpt_valid = false; ++c->state_gen;
    clear_final_marks(c);
    RC(stage_h2d(c, vec_dest(c->d_ckpt, c->pvec, 4), (const uint8_t*)ckpt, bytes, is_pinned(ckpt)));
    c->ckpt_valid = true; ++c->state_gen;
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
    CK(c, hipStreamSynchronize(c->stream));
    return PGH_OK;
}

}  // extern "C"

// ---- internals for the multi-GPU group driver (pgh_internal.h) ------------------------------------

namespace pgh_int {
bool peek_valid(const pgh_ctx* c) { return c->peek_gen != 0 && c->peek_gen == c->state_gen; }

void peek_wait(pgh_ctx* c) { peek_job_wait(c); }

int peek_commit(pgh_ctx* c, const uint8_t* out_frame, size_t n, uint8_t* out) {
    std::vector<std::pair<size_t, size_t>> spans;
    RC(state_shard_spans(c, out_frame, n, &spans, "peeked checkpoint frame"));
    DeviceGuard g(c->device);
    peek_job_wait(c);
    bool copied;
    {
        std::lock_guard<std::mutex> lk(c->pk_mu);
        copied = c->pk_done_gen == c->peek_gen && c->pk_done_out == out;
    }
    clear_final_marks(c);  // they describe the fold that wrote the old checkpoint buffer
    if (copied) {  // the peek thread already put this peek's payloads into `out`
        std::swap(c->d_ckpt, c->d_peek);
        c->acc_src = nullptr;
        c->folded = 0;
        c->st.n_folded = 0;
        c->slot_mode = -1;
        c->peek_gen = 0;
        ++c->state_gen;
        return PGH_OK;
    }
    CK(c, hipEventSynchronize(c->peek_ev));
    std::vector<OutPiece> pieces;
    size_t total = 0;
    for (auto& sp : spans) {
        pieces.push_back(OutPiece{out + sp.first, sp.second});
        total += sp.second;
    }
    if (total != (size_t)c->pg * 4) return fail(c, PGH_E_ARG, "frame holds %zu payload bytes of this shard, %lld expected",
                                                 total, (long long)c->pg * 4);
    scatter_out((const uint8_t*)c->h_peek, 0, total, pieces, *c->pool_copy);
    std::swap(c->d_ckpt, c->d_peek);  // the peeked result IS the new checkpoint, as after a FINAL fold
    c->acc_src = nullptr;
    c->folded = 0;
    c->st.n_folded = 0;
    c->slot_mode = -1;
    c->peek_gen = 0;
    ++c->state_gen;
    return PGH_OK;
}


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
int64_t shard_lo(const pgh_ctx* c) { return c->lo; }
int64_t shard_len(const pgh_ctx* c) { return c->pg; }
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
    peek_job_wait(c);  // a peek's payload copy may still be writing the same output
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

