// libpygrid_hip: C-ABI context around the gfx950 aggregation kernels.
//
// One pgh_ctx = one GPU = one parameter shard.  It owns
//   * the HBM slab [max_clients x rows_per_client][ld] holding every reported diff of the
//     cycle (fp32) or every share (int64), rows padded to 256 B,
//   * the [P_shard] device vectors (checkpoint, output, running state, weights),
//   * a 2-slot pinned host ring through which ingest streams host bytes into the slab with
//     hipMemcpyAsync on a dedicated copy stream (overlapping the next slot's host memcpy),
//   * HIP event pairs around every reduction launch (pgh_stats reports kernel time).
//
// Reference mapping: ingest = the N x unserialize_model_params loop of
// cycle_manager.py:247-250; pgh_fedavg = :252-296; pgh_secagg = PySyft share add + .get() +
// float_prec (test_basic_syft_operations.py:417-424).  Errors map to negative status codes and
// a message (the Python shim raises a PyGridError subclass, as tasks/cycle.py:33-37 expects).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pgh_api.h"
#include "pgh_kernels.h"
#include "pgh_state.h"

struct pgh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // reductions
    hipStream_t copy = nullptr;    // ingest H2D
    hipEvent_t copy_done = nullptr;

    std::vector<int64_t> numel;
    int64_t P = 0, lo = 0, hi = 0, pg = 0, ld = 0;
    bool layout = false;

    int max_clients = 0, dtype = PGH_F32, parties = 1;
    void* d_slab = nullptr;
    size_t slab_bytes = 0;
    size_t vec_cap = 0;  // elements of each [P_shard] vector (= ld)
    float* d_ckpt = nullptr;
    float* d_out = nullptr;
    float* d_acc = nullptr;
    uint64_t* d_uacc = nullptr;
    int64_t* d_sum = nullptr;
    float* d_dec = nullptr;
    float* d_w = nullptr;

    uint8_t* h_pin[2] = {nullptr, nullptr};
    size_t pin_slot = 0;
    hipEvent_t pin_ev[2] = {nullptr, nullptr};
    bool pin_used[2] = {false, false};
    int pin_next = 0;

    std::vector<uint8_t> have;
    std::vector<float> weights;
    int variant = 0;

    struct Timed { hipEvent_t a, b; uint64_t bytes; };
    std::vector<Timed> pending;
    std::vector<hipEvent_t> pool;
    pgh_stats_t st{};
    std::vector<float> scratch;  // State decode staging
    std::string err;
};

namespace {

thread_local std::string g_create_err;

int fail(pgh_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf; else g_create_err = buf;
    return code;
}

#define CK(c, expr)                                                                        \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail((c), PGH_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                               \
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

void free_slab(pgh_ctx* c) {
    (void)hipDeviceSynchronize();
    (void)hipFree(c->d_slab); c->d_slab = nullptr; c->slab_bytes = 0;
    (void)hipFree(c->d_ckpt); c->d_ckpt = nullptr;
    (void)hipFree(c->d_out); c->d_out = nullptr;
    (void)hipFree(c->d_acc); c->d_acc = nullptr;
    (void)hipFree(c->d_uacc); c->d_uacc = nullptr;
    (void)hipFree(c->d_sum); c->d_sum = nullptr;
    (void)hipFree(c->d_dec); c->d_dec = nullptr;
    (void)hipFree(c->d_w); c->d_w = nullptr;
    c->vec_cap = 0;
    c->max_clients = 0;
    c->have.clear();
}

// Clients ingested must be exactly {0..n-1}: the fold order is the client order.
int contiguous_clients(pgh_ctx* c, int* n_out) {
    int n = 0;
    while (n < (int)c->have.size() && c->have[n]) ++n;
    for (int k = n; k < (int)c->have.size(); ++k)
        if (c->have[k]) return fail(c, PGH_E_STATE, "client %d is missing but client %d was ingested", n, k);
    if (n == 0) return fail(c, PGH_E_STATE, "no diffs ingested");
    *n_out = n;
    return PGH_OK;
}

int check_ready(pgh_ctx* c, int dtype) {
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (!c->d_slab) return fail(c, PGH_E_STATE, "pgh_reserve has not been called");
    if (c->dtype != dtype)
        return fail(c, PGH_E_STATE, "slab holds dtype %d, call needs %d", c->dtype, dtype);
    return PGH_OK;
}

hipEvent_t take_event(pgh_ctx* c) {
    if (!c->pool.empty()) { hipEvent_t e = c->pool.back(); c->pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int collect_timings(pgh_ctx* c) {
    for (auto& t : c->pending) {
        CK(c, hipEventSynchronize(t.b));
        float ms = 0.f;
        CK(c, hipEventElapsedTime(&ms, t.a, t.b));
        c->st.kernel_ms_last = ms;
        c->st.kernel_ms_total += ms;
        c->st.kernel_launches += 1;
        c->st.kernel_bytes_last = t.bytes;
        c->pool.push_back(t.a);
        c->pool.push_back(t.b);
    }
    c->pending.clear();
    return PGH_OK;
}

// Bracket a launch with an event pair on `s`.
template <class F>
int timed_launch(pgh_ctx* c, hipStream_t s, uint64_t bytes, F&& launch) {
    if (c->pending.size() >= 4096) {
        int rc = collect_timings(c);
        if (rc) return rc;
    }
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

// host -> HBM through the pinned ring on the copy stream
int stage_h2d(pgh_ctx* c, void* dst, const uint8_t* src, size_t n) {
    const double t0 = now_ms();
    size_t off = 0;
    while (off < n) {
        const int slot = c->pin_next;
        c->pin_next ^= 1;
        if (c->pin_used[slot]) CK(c, hipEventSynchronize(c->pin_ev[slot]));
        const size_t m = (n - off < c->pin_slot) ? (n - off) : c->pin_slot;
        std::memcpy(c->h_pin[slot], src + off, m);
        CK(c, hipMemcpyAsync((uint8_t*)dst + off, c->h_pin[slot], m, hipMemcpyHostToDevice, c->copy));
        CK(c, hipEventRecord(c->pin_ev[slot], c->copy));
        c->pin_used[slot] = true;
        off += m;
    }
    c->st.h2d_ms_total += now_ms() - t0;
    c->st.h2d_bytes_total += n;
    return PGH_OK;
}

// The reduction stream waits for every ingest copy issued so far.
int order_after_ingest(pgh_ctx* c, hipStream_t s) {
    CK(c, hipEventRecord(c->copy_done, c->copy));
    CK(c, hipStreamWaitEvent(s, c->copy_done, 0));
    return PGH_OK;
}

int run_fedavg(pgh_ctx* c, int mode, const float* d_ckpt, float* d_out, hipStream_t s) {
    int n = 0;
    int rc = contiguous_clients(c, &n);
    if (rc) return rc;
    if (mode != PGH_MEAN && mode != PGH_ITERATIVE_MEAN && mode != PGH_WEIGHTED_MEAN)
        return fail(c, PGH_E_ARG, "unknown averaging mode %d", mode);
    float divisor = (float)n;  // th.div(sum, len(diffs)), cycle_manager.py:288
    if (mode == PGH_WEIGHTED_MEAN) {
        if ((int)c->weights.size() != n)
            return fail(c, PGH_E_STATE, "weighted mean needs %d weights, have %zu", n, c->weights.size());
        float t = c->weights[0];
        for (int k = 1; k < n; ++k) t = t + c->weights[k];  // left fold, float32
        if (!(t != 0.f)) return fail(c, PGH_E_ARG, "sum of weights is zero");
        divisor = t;
        CK(c, hipMemcpyAsync(c->d_w, c->weights.data(), sizeof(float) * n, hipMemcpyHostToDevice, s));
    }
    rc = order_after_ingest(c, s);
    if (rc) return rc;
    pgh::FedavgArgs a{};
    a.diffs = (const float*)c->d_slab;
    a.ld = c->ld;
    a.n_rows = n;
    a.client0 = 0;
    a.p = c->pg;
    a.weights = c->d_w;
    a.acc = c->d_acc;
    a.ckpt = d_ckpt;
    a.out = d_out;
    a.divisor = divisor;
    a.flags = pgh::FL_FIRST | pgh::FL_FINAL;
    a.mode = mode;
    a.variant = c->variant;
    const uint64_t bytes = 4ull * (uint64_t)n * (uint64_t)c->pg + 8ull * (uint64_t)c->pg;
    return timed_launch(c, s, bytes, [&] { return pgh::launch_fedavg(a, s); });
}

int run_secagg(pgh_ctx* c, int base, int prec, int64_t* d_sum, float* d_dec, hipStream_t s) {
    int n = 0;
    int rc = contiguous_clients(c, &n);
    if (rc) return rc;
    if (base < 2 || prec < 0 || prec > 18) return fail(c, PGH_E_ARG, "bad fixed-point base %d / precision %d", base, prec);
    long double scale = 1;
    for (int k = 0; k < prec; ++k) scale *= base;
    if (scale > 9.2e18L) return fail(c, PGH_E_ARG, "base**prec overflows int64");
    rc = order_after_ingest(c, s);
    if (rc) return rc;
    pgh::SecaggArgs a{};
    a.shares = (const int64_t*)c->d_slab;
    a.ld = c->ld;
    a.n_rows = n * c->parties;
    a.p = c->pg;
    a.acc = c->d_uacc;
    a.sum_out = d_sum;
    a.dec_out = d_dec;
    a.divisor = (float)(int64_t)scale;  // python int base**prec, promoted to float32
    a.flags = pgh::FL_FIRST | pgh::FL_FINAL;
    a.variant = c->variant;
    const uint64_t bytes = 8ull * (uint64_t)a.n_rows * (uint64_t)c->pg + (d_sum ? 8ull * c->pg : 0) +
                           (d_dec ? 4ull * c->pg : 0);
    return timed_launch(c, s, bytes, [&] { return pgh::launch_secagg(a, s); });
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
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&c->copy_done, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->pin_ev[0], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->pin_ev[1], hipEventDisableTiming) == hipSuccess;
    if (!ok) { pgh_destroy(c); return fail(nullptr, PGH_E_HIP, "stream/event creation failed"); }
    for (int k = 0; k < 2; ++k)
        if (hipHostMalloc((void**)&c->h_pin[k], c->pin_slot, hipHostMallocDefault) != hipSuccess) {
            pgh_destroy(c);
            return fail(nullptr, PGH_E_OOM, "pinned host allocation of %zu bytes failed", c->pin_slot);
        }
    *out = c;
    return PGH_OK;
}

void pgh_destroy(pgh_ctx* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    free_slab(c);
    for (auto& t : c->pending) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    for (int k = 0; k < 2; ++k) {
        if (c->h_pin[k]) (void)hipHostFree(c->h_pin[k]);
        if (c->pin_ev[k]) (void)hipEventDestroy(c->pin_ev[k]);
    }
    if (c->copy_done) (void)hipEventDestroy(c->copy_done);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    delete c;
}

int pgh_set_layout(pgh_ctx* c, int n_tensors, const int64_t* numel) {
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
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (lo < 0 || hi > c->P || lo >= hi) return fail(c, PGH_E_ARG, "shard [%lld,%lld) outside [0,%lld)",
                                                    (long long)lo, (long long)hi, (long long)c->P);
    DeviceGuard g(c->device);
    free_slab(c);
    c->lo = lo;
    c->hi = hi;
    c->pg = hi - lo;
    c->ld = (c->pg + 63) & ~(int64_t)63;  // 256-B (fp32) / 512-B (int64) row pitch
    c->st.p_shard = c->pg;
    c->st.ld = c->ld;
    return PGH_OK;
}

int pgh_reserve(pgh_ctx* c, int max_clients, int dtype, int n_parties) {
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (max_clients <= 0) return fail(c, PGH_E_ARG, "max_clients must be positive");
    if (dtype != PGH_F32 && dtype != PGH_I64) return fail(c, PGH_E_ARG, "unknown dtype %d", dtype);
    if (dtype == PGH_F32) n_parties = 1;
    if (n_parties < 1) return fail(c, PGH_E_ARG, "n_parties must be >= 1");
    DeviceGuard g(c->device);
    free_slab(c);
    const size_t esz = dtype == PGH_F32 ? 4 : 8;
    const size_t rows = (size_t)max_clients * (size_t)n_parties;
    const size_t bytes = rows * (size_t)c->ld * esz;
    if (hipMalloc(&c->d_slab, bytes) != hipSuccess) {
        c->d_slab = nullptr;
        (void)hipGetLastError();
        return fail(c, PGH_E_OOM, "slab allocation of %zu bytes (%zu rows x %lld) failed", bytes, rows, (long long)c->ld);
    }
    c->slab_bytes = bytes;
    c->vec_cap = (size_t)c->ld;
    const size_t v4 = c->vec_cap * 4, v8 = c->vec_cap * 8;
    bool ok = hipMalloc((void**)&c->d_ckpt, v4) == hipSuccess && hipMalloc((void**)&c->d_out, v4) == hipSuccess &&
              hipMalloc((void**)&c->d_acc, v4) == hipSuccess && hipMalloc((void**)&c->d_uacc, v8) == hipSuccess &&
              hipMalloc((void**)&c->d_sum, v8) == hipSuccess && hipMalloc((void**)&c->d_dec, v4) == hipSuccess &&
              hipMalloc((void**)&c->d_w, sizeof(float) * (size_t)max_clients) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        free_slab(c);
        return fail(c, PGH_E_OOM, "device vector allocation failed");
    }
    c->max_clients = max_clients;
    c->dtype = dtype;
    c->parties = n_parties;
    c->have.assign((size_t)max_clients, 0);
    c->weights.clear();
    c->st.max_clients = max_clients;
    c->st.n_clients = 0;
    return PGH_OK;
}

int pgh_reset(pgh_ctx* c) {
    if (!c) return PGH_E_ARG;
    std::fill(c->have.begin(), c->have.end(), 0);
    c->weights.clear();
    c->st.n_clients = 0;
    return PGH_OK;
}

int pgh_ingest_raw(pgh_ctx* c, int client, const void* flat, size_t nbytes, int dtype) {
    int rc = check_ready(c, dtype);
    if (rc) return rc;
    if (!flat) return fail(c, PGH_E_ARG, "flat is NULL");
    if (client < 0 || client >= c->max_clients)
        return fail(c, PGH_E_ARG, "client %d outside slab capacity %d", client, c->max_clients);
    const size_t esz = dtype == PGH_F32 ? 4 : 8;
    const size_t want = (size_t)c->P * esz * (size_t)c->parties;
    if (nbytes != want) return fail(c, PGH_E_ARG, "client %d: got %zu bytes, layout needs %zu", client, nbytes, want);
    DeviceGuard g(c->device);
    const uint8_t* src = (const uint8_t*)flat;
    for (int s = 0; s < c->parties; ++s) {
        const size_t row = (size_t)client * c->parties + s;
        uint8_t* dst = (uint8_t*)c->d_slab + row * (size_t)c->ld * esz;
        rc = stage_h2d(c, dst, src + ((size_t)s * c->P + c->lo) * esz, (size_t)c->pg * esz);
        if (rc) return rc;
    }
    if (!c->have[client]) c->st.n_clients += 1;
    c->have[client] = 1;
    return PGH_OK;
}

int pgh_ingest_state(pgh_ctx* c, int client, const uint8_t* pb, size_t n) {
    int rc = check_ready(c, PGH_F32);
    if (rc) return rc;
    if (!pb && n) return fail(c, PGH_E_ARG, "pb is NULL");
    if (client < 0 || client >= c->max_clients)
        return fail(c, PGH_E_ARG, "client %d outside slab capacity %d", client, c->max_clients);
    c->scratch.resize((size_t)c->P);
    std::string msg;
    rc = pgh_state::decode_f32(pb, n, c->numel, c->scratch.data(), &msg);
    if (rc) return fail(c, rc, "client %d State: %s", client, msg.c_str());
    return pgh_ingest_raw(c, client, c->scratch.data(), (size_t)c->P * 4, PGH_F32);
}

int pgh_synth_fill(pgh_ctx* c, uint64_t seed, int n_clients) {
    int rc = check_ready(c, c ? c->dtype : 0);
    if (rc) return rc;
    if (n_clients <= 0 || n_clients > c->max_clients)
        return fail(c, PGH_E_ARG, "n_clients %d outside (0,%d]", n_clients, c->max_clients);
    DeviceGuard g(c->device);
    hipError_t e;
    if (c->dtype == PGH_F32)
        e = pgh::launch_synth_f32((float*)c->d_slab, n_clients, c->ld, c->pg, seed, pgh::STREAM_DIFF, 0, c->lo,
                                  pgh::DIFF_SCALE, c->copy);
    else
        e = pgh::launch_synth_shares((int64_t*)c->d_slab, n_clients, c->parties, c->ld, c->pg, seed, 0, c->lo,
                                     1000.0f, c->copy);
    if (e != hipSuccess) return fail(c, PGH_E_HIP, "synthetic fill failed: %s", hipGetErrorString(e));
    for (int k = 0; k < n_clients; ++k) c->have[k] = 1;
    for (int k = n_clients; k < c->max_clients; ++k) c->have[k] = 0;
    c->st.n_clients = n_clients;
    return PGH_OK;
}

int pgh_synth_ckpt_device(pgh_ctx* c, uint64_t seed, float* d_ckpt, void* stream) {
    if (!c) return PGH_E_ARG;
    if (!c->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (!d_ckpt) return fail(c, PGH_E_ARG, "d_ckpt is NULL");
    DeviceGuard g(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // one row of exactly P_shard elements (ld = P_shard rounded to 4 would overrun the buffer)
    if (c->pg % 4 == 0) {
        hipError_t e = pgh::launch_synth_f32(d_ckpt, 1, c->pg, c->pg, seed, pgh::STREAM_CKPT, 0, c->lo,
                                             pgh::CKPT_SCALE, s);
        if (e != hipSuccess) return fail(c, PGH_E_HIP, "synthetic checkpoint failed: %s", hipGetErrorString(e));
        return PGH_OK;
    }
    if (!c->d_ckpt) return fail(c, PGH_E_STATE, "pgh_reserve has not been called");
    hipError_t e = pgh::launch_synth_f32(c->d_ckpt, 1, c->ld, c->pg, seed, pgh::STREAM_CKPT, 0, c->lo,
                                         pgh::CKPT_SCALE, s);
    if (e != hipSuccess) return fail(c, PGH_E_HIP, "synthetic checkpoint failed: %s", hipGetErrorString(e));
    CK(c, hipMemcpyAsync(d_ckpt, c->d_ckpt, sizeof(float) * c->pg, hipMemcpyDeviceToDevice, s));
    return PGH_OK;
}

int pgh_set_weights(pgh_ctx* c, const float* w, int n) {
    if (!c) return PGH_E_ARG;
    if (!w || n <= 0) return fail(c, PGH_E_ARG, "need a non-empty weight vector");
    if (n > c->max_clients) return fail(c, PGH_E_ARG, "%d weights for a %d-client slab", n, c->max_clients);
    c->weights.assign(w, w + n);
    return PGH_OK;
}

int pgh_fedavg_device(pgh_ctx* c, int mode, const float* d_ckpt, float* d_out, void* stream) {
    int rc = check_ready(c, PGH_F32);
    if (rc) return rc;
    if (!d_ckpt || !d_out) return fail(c, PGH_E_ARG, "d_ckpt / d_out is NULL");
    if (((uintptr_t)d_ckpt | (uintptr_t)d_out) & 15) return fail(c, PGH_E_ARG, "device buffers must be 16-byte aligned");
    DeviceGuard g(c->device);
    return run_fedavg(c, mode, d_ckpt, d_out, stream ? (hipStream_t)stream : c->stream);
}

int pgh_fedavg(pgh_ctx* c, int mode, const float* ckpt, float* out) {
    int rc = check_ready(c, PGH_F32);
    if (rc) return rc;
    if (!ckpt || !out) return fail(c, PGH_E_ARG, "ckpt / out is NULL");
    DeviceGuard g(c->device);
    const double t0 = now_ms();
    const size_t bytes = sizeof(float) * (size_t)c->pg;
    CK(c, hipMemcpyAsync(c->d_ckpt, ckpt, bytes, hipMemcpyHostToDevice, c->stream));
    rc = run_fedavg(c, mode, c->d_ckpt, c->d_out, c->stream);
    if (rc) return rc;
    CK(c, hipMemcpyAsync(out, c->d_out, bytes, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->st.close_ms_last = now_ms() - t0;
    return collect_timings(c);
}

int pgh_secagg_device(pgh_ctx* c, int base, int prec, int64_t* d_sum, float* d_dec, void* stream) {
    int rc = check_ready(c, PGH_I64);
    if (rc) return rc;
    DeviceGuard g(c->device);
    return run_secagg(c, base, prec, d_sum, d_dec, stream ? (hipStream_t)stream : c->stream);
}

int pgh_secagg(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out) {
    int rc = check_ready(c, PGH_I64);
    if (rc) return rc;
    DeviceGuard g(c->device);
    const double t0 = now_ms();
    rc = run_secagg(c, base, prec, sum_out ? c->d_sum : nullptr, dec_out ? c->d_dec : nullptr, c->stream);
    if (rc) return rc;
    if (sum_out) CK(c, hipMemcpyAsync(sum_out, c->d_sum, 8ull * c->pg, hipMemcpyDeviceToHost, c->stream));
    if (dec_out) CK(c, hipMemcpyAsync(dec_out, c->d_dec, 4ull * c->pg, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->st.close_ms_last = now_ms() - t0;
    return collect_timings(c);
}

int pgh_set_variant(pgh_ctx* c, int variant) {
    if (!c) return PGH_E_ARG;
    if (variant < 0 || variant > 5) return fail(c, PGH_E_ARG, "variant %d outside [0,5]", variant);
    c->variant = variant;
    return PGH_OK;
}

int pgh_stats(pgh_ctx* c, pgh_stats_t* out) {
    if (!c || !out) return PGH_E_ARG;
    DeviceGuard g(c->device);
    int rc = collect_timings(c);
    if (rc) return rc;
    *out = c->st;
    return PGH_OK;
}

int pgh_reset_stats(pgh_ctx* c) {
    if (!c) return PGH_E_ARG;
    DeviceGuard g(c->device);
    int rc = collect_timings(c);
    if (rc) return rc;
    const int64_t pg = c->st.p_shard, ld = c->st.ld;
    const int32_t n = c->st.n_clients, m = c->st.max_clients;
    c->st = pgh_stats_t{};
    c->st.p_shard = pg; c->st.ld = ld; c->st.n_clients = n; c->st.max_clients = m;
    return PGH_OK;
}

int pgh_slab(pgh_ctx* c, void** d_slab, int64_t* ld) {
    if (!c || !d_slab || !ld) return PGH_E_ARG;
    *d_slab = c->d_slab;
    *ld = c->ld;
    return PGH_OK;
}

}  // extern "C"
