// libpygrid_hip multi-GPU group: one context over the GPUs of one node, in ONE process.
//
// PyGrid Node closes a cycle from a single Flask-Executor thread in a single process
// (apps/node/src/app/__init__.py:196-199, tasks/cycle.py:9-25, sole caller
// cycle_manager.py:217), so the drop-in cannot rely on one process per GPU: the library itself
// drives every GPU.  pgh_create_group builds one child context per device (pgh_create) plus
//   * a fan-out pool with one host thread per GPU (the caller's thread serves GPU 0), so every
//     call stages each GPU's bytes over that GPU's own PCIe link and launches its kernels at once;
//   * the exchange between GPUs: RCCL communicators over all devices (ncclCommInitAll; librccl is
//     dlopen'ed at first use, so the library has no link-time RCCL dependency and shares the copy
//     torch already loaded), or peer copies when the devices are not distinct / PGH_RCCL=0.
//
// Partition.  The group's parameter range is cut into contiguous shards of S
// elements (ceil(len / G) rounded up to 64), one per GPU; every GPU holds every client for its
// shard, so each shard folds the clients in the reference's order and the fp32 result is bit-
// identical to one GPU.  Host outputs are written slice by slice (no collective needed); the
// resident checkpoint can be all-gathered into a full copy on every GPU (ncclAllGather).
// Secure aggregation can shard the CLIENTS instead (pgh_set_client_sharding): GPU g holds clients
// [g * per, (g + 1) * per) over the whole model, sums them (K3, no decode), the Z_2^64 sums are
// reduce-scattered (ncclReduceScatter, uint64 SUM: wrap-add is associative, so exact), and GPU g
// decodes its slice -- the layout when each GPU ingests its own clients over its own link.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pgh_api.h"
#include "pgh_internal.h"
#include "pgh_kernels.h"
#include "pgh_state.h"

namespace {

// One persistent host thread per child but the first (run on the caller's thread): run(f) calls
// f(i) for every child i concurrently and returns when all are done.
class Fanout {
  public:
    explicit Fanout(int n) : n_(n) {
        for (int t = 1; t < n_; ++t) workers_.emplace_back([this, t] { loop(t); });
    }
    ~Fanout() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    void run(const std::function<void(int)>& f) {
        if (n_ == 1) { f(0); return; }
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &f;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

  private:
    void loop(int t) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* fn;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                fn = fn_;
            }
            (*fn)(t);
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// The RCCL entry points the group uses, resolved from librccl.so.1 at first use.
struct Rccl {
    void* h = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
};

const Rccl* load_rccl(std::string* why) {
    static Rccl r;
    static std::string err;
    static std::once_flag once;
    std::call_once(once, [] {
        // the copy torch loaded (same soname) if it is in the process, else the ROCm install's
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (r.h) break;
        }
        if (!r.h) { err = std::string("cannot load librccl.so.1: ") + dlerror(); return; }
        r.comm_init_all = (decltype(r.comm_init_all))dlsym(r.h, "ncclCommInitAll");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
        r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
        r.group_start = (decltype(r.group_start))dlsym(r.h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(r.h, "ncclGroupEnd");
        r.all_gather = (decltype(r.all_gather))dlsym(r.h, "ncclAllGather");
        r.reduce_scatter = (decltype(r.reduce_scatter))dlsym(r.h, "ncclReduceScatter");
        if (!r.comm_init_all || !r.comm_destroy || !r.error_string || !r.group_start || !r.group_end ||
            !r.all_gather || !r.reduce_scatter) {
            err = "librccl.so.1 lacks an entry point the group needs";
            r.h = nullptr;
        }
    });
    if (!r.h) {
        if (why) *why = err;
        return nullptr;
    }
    return &r;
}

constexpr int64_t ALIGN = 64;  // shard starts stay 256-byte aligned (pygrid_amd/sharding.py ALIGN)

int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct pgh_group {
    std::vector<pgh_ctx*> kids;
    std::vector<int> devs;
    std::unique_ptr<Fanout> fan;
    std::vector<int64_t> numel;
    bool layout = false;
    int64_t P = 0, lo = 0, hi = 0;
    int64_t S = 0;            // shard length of every GPU (the last may hold fewer real params)
    int active = 0;           // GPUs holding a non-empty param shard (all of them unless P is tiny)
    bool want_client_shard = false;
    bool client_shard = false;  // the reserved slab is client-sharded (int64 secagg)
    int per = 0;              // clients per GPU when client-sharded
    int dtype = PGH_F32, parties = 1, max_clients = 0;
    std::vector<int> kid_clients;  // client-sharded: clients ingested per GPU since the last reset
    std::vector<std::vector<char>> kid_seen;
    // exchange
    int backend = -1;         // -1 not chosen yet, 1 RCCL, 0 peer copies
    int comm_n = 0;           // GPUs in `comms`
    std::vector<ncclComm_t> comms;
    const Rccl* rccl = nullptr;
    std::vector<void*> d_full;   // all-gather destination per GPU: G x S floats
    std::vector<void*> d_rs;     // client-sharded secagg: this GPU's reduced slice (S int64)
    std::vector<void*> d_stage;  // peer-copy reduce-scatter staging: G x S int64 per GPU
    int64_t full_cap = 0, rs_cap = 0, stage_cap = 0;
};

namespace {

using pgh_int::fail;

pgh_group* G(pgh_ctx* c) { return pgh_int::group_of(c); }

// Run f on every child in `n` (default: the active ones) concurrently; the first failure's
// message becomes the group's, prefixed with the GPU.
int fan(pgh_ctx* c, const std::function<int(int, pgh_ctx*)>& f, int n = -1) {
    pgh_group* g = G(c);
    if (n < 0) n = g->active;
    std::vector<int> rc((size_t)g->kids.size(), PGH_OK);
    g->fan->run([&](int i) {
        if (i < n) rc[(size_t)i] = f(i, g->kids[(size_t)i]);
    });
    for (int i = 0; i < n; ++i)
        if (rc[(size_t)i] != PGH_OK)
            return fail(c, rc[(size_t)i], "gpu %d (device %d): %s", i, g->devs[(size_t)i],
                        pgh_last_error(g->kids[(size_t)i]));
    return PGH_OK;
}

int need_layout(pgh_ctx* c) {
    if (!G(c)->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    return PGH_OK;
}

int need_slab(pgh_ctx* c) {
    if (!G(c)->layout) return fail(c, PGH_E_STATE, "pgh_set_layout has not been called");
    if (G(c)->max_clients <= 0) return fail(c, PGH_E_STATE, "pgh_reserve has not been called");
    return PGH_OK;
}

#define RC(expr)            \
    do {                    \
        int r_ = (expr);    \
        if (r_) return r_;  \
    } while (0)

// Param shards of [lo, hi) over the GPUs: S per GPU, 64-aligned; a tiny model uses fewer GPUs.
int plan_shards(pgh_ctx* c) {
    pgh_group* g = G(c);
    const int n = (int)g->kids.size();
    const int64_t len = g->hi - g->lo;
    g->S = round_up((len + n - 1) / n, ALIGN);
    g->active = (int)std::min<int64_t>(n, (len + g->S - 1) / g->S);
    return PGH_OK;
}

int64_t kid_lo(const pgh_group* g, int i) { return g->lo + (int64_t)i * g->S; }
int64_t kid_hi(const pgh_group* g, int i) { return std::min(g->hi, g->lo + (int64_t)(i + 1) * g->S); }

// Lay the children out: param shards (default) or, client-sharded, the whole range on every GPU.
int apply_shards(pgh_ctx* c, bool client_shard) {
    pgh_group* g = G(c);
    RC(plan_shards(c));
    if (client_shard) {
        const int n = (int)g->kids.size();
        g->active = n;
        return fan(c, [&](int, pgh_ctx* k) -> int {
            RC(pgh_int::set_vec_min(k, (int64_t)n * g->S));  // the reduce-scatter's send buffer: G x S
            return pgh_set_shard(k, g->lo, g->hi);
        }, n);
    }
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        RC(pgh_int::set_client_base(k, 0));
        RC(pgh_int::set_vec_min(k, g->S));  // all-gather: equal padded shards
        return pgh_set_shard(k, kid_lo(g, i), kid_hi(g, i));
    });
}

float fixed_point_divisor(int base, int prec) {
    long double scale = 1;
    for (int k = 0; k < prec; ++k) scale *= base;
    return (float)(int64_t)scale;
}

struct DevSel {  // select a device for this thread, restore the previous one after
    int prev = -1;
    explicit DevSel(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(d);
    }
    ~DevSel() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int free_exchange(pgh_group* g) {
    for (size_t i = 0; i < g->kids.size(); ++i) {
        DevSel d(g->devs[i]);
        if (i < g->d_full.size()) (void)hipFree(g->d_full[i]);
        if (i < g->d_rs.size()) (void)hipFree(g->d_rs[i]);
        if (i < g->d_stage.size()) (void)hipFree(g->d_stage[i]);
    }
    g->d_full.clear();
    g->d_rs.clear();
    g->d_stage.clear();
    g->full_cap = g->rs_cap = g->stage_cap = 0;
    return PGH_OK;
}

// Choose RCCL or peer copies for the active GPUs (once per set of GPUs).
int ensure_backend(pgh_ctx* c, int n) {
    pgh_group* g = G(c);
    if (g->backend >= 0 && g->comm_n == n) return PGH_OK;
    if (g->rccl) {
        for (auto cm : g->comms) g->rccl->comm_destroy(cm);
    }
    g->comms.clear();
    g->comm_n = n;
    std::vector<int> devs(g->devs.begin(), g->devs.begin() + n);
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const char* env = std::getenv("PGH_RCCL");
    const bool allowed = !env || std::atoi(env) != 0;
    g->backend = 0;
    if (distinct && allowed && n >= 1) {
        std::string why;
        const Rccl* r = load_rccl(&why);
        if (r) {
            g->rccl = r;
            g->comms.assign((size_t)n, nullptr);
            int cur = 0;
            (void)hipGetDevice(&cur);
            DevSel keep(cur);  // the caller's current device survives the communicator setup
            const ncclResult_t e = r->comm_init_all(g->comms.data(), n, devs.data());
            if (e != ncclSuccess) {
                g->comms.clear();
                g->backend = -1;  // not silently peer copies: the next collective tries RCCL again (and fails loudly)
                g->comm_n = 0;
                return fail(c, PGH_E_HIP, "ncclCommInitAll over %d GPUs failed: %s", n, r->error_string(e));
            }
            g->backend = 1;
        }
    }
    return PGH_OK;
}

int grow(pgh_ctx* c, std::vector<void*>* bufs, int64_t* cap, int64_t bytes) {
    pgh_group* g = G(c);
    if ((int64_t)bufs->size() == (int64_t)g->kids.size() && *cap >= bytes) return PGH_OK;
    for (size_t i = 0; i < bufs->size(); ++i) {
        DevSel d(g->devs[i]);
        (void)hipFree((*bufs)[i]);
    }
    bufs->assign(g->kids.size(), nullptr);
    *cap = 0;
    for (size_t i = 0; i < g->kids.size(); ++i) {
        DevSel d(g->devs[i]);
        if (hipMalloc(&(*bufs)[i], (size_t)bytes) != hipSuccess) {
            (void)hipGetLastError();
            return fail(c, PGH_E_OOM, "gpu %zu: exchange buffer of %lld bytes failed", i, (long long)bytes);
        }
    }
    *cap = bytes;
    return PGH_OK;
}

int sync_all(pgh_ctx* c, int n) {
    return fan(c, [](int, pgh_ctx* k) -> int { return pgh_sync(k); }, n);
}

// Client-sharded secure aggregation: per-GPU share sums -> reduce-scatter -> per-GPU decode ->
// host slices.
int secagg_client_sharded(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out) {
    pgh_group* g = G(c);
    const int n = (int)g->kids.size();
    const int64_t S = g->S, L = (int64_t)n * S, len = g->hi - g->lo;
    int total = 0;
    for (int v : g->kid_clients) total += v;
    if (total == 0) return fail(c, PGH_E_STATE, "no diffs ingested");
    if (base < 2 || prec < 0 || prec > 18) return fail(c, PGH_E_ARG, "bad fixed-point base %d / precision %d", base, prec);
    // 1. every GPU sums its own clients over the whole range (zeros if it holds none); the tail
    //    [len, L) of the send buffer stays zero so the padded slices reduce to zero
    RC(fan(c, [&](int i, pgh_ctx* k) -> int {
        DevSel d(pgh_int::device_of(k));
        int64_t* d_sum = (int64_t*)pgh_int::vec(k, pgh_int::V_SUM);
        const hipStream_t s = pgh_int::stream_of(k);
        if (hipMemsetAsync(d_sum + len, 0, (size_t)(L - len) * 8, s) != hipSuccess)
            return pgh_int::fail(k, PGH_E_HIP, "memset of the padded share-sum tail failed");
        if (g->kid_clients[(size_t)i] == 0) {
            if (hipMemsetAsync(d_sum, 0, (size_t)len * 8, s) != hipSuccess)
                return pgh_int::fail(k, PGH_E_HIP, "memset of an empty GPU's share sum failed");
            return PGH_OK;
        }
        return pgh_secagg_device(k, base, prec, d_sum, nullptr, s);
    }, n));
    RC(ensure_backend(c, n));
    RC(grow(c, &g->d_rs, &g->rs_cap, S * 8));
    const float div = fixed_point_divisor(base, prec);
    if (g->backend == 1) {
        // 2. reduce-scatter over RCCL: GPU i receives the Z_2^64 total of slice i
        g->rccl->group_start();
        for (int i = 0; i < n; ++i) {
            pgh_ctx* k = g->kids[(size_t)i];
            DevSel d(pgh_int::device_of(k));
            const ncclResult_t e = g->rccl->reduce_scatter(pgh_int::vec(k, pgh_int::V_SUM), g->d_rs[(size_t)i],
                                                           (size_t)S, ncclUint64, ncclSum, g->comms[(size_t)i],
                                                           pgh_int::stream_of(k));
            if (e != ncclSuccess) {
                g->rccl->group_end();
                return fail(c, PGH_E_HIP, "ncclReduceScatter on gpu %d failed: %s", i, g->rccl->error_string(e));
            }
        }
        const ncclResult_t e = g->rccl->group_end();
        if (e != ncclSuccess) return fail(c, PGH_E_HIP, "ncclGroupEnd failed: %s", g->rccl->error_string(e));
        // 3. each GPU decodes its slice (the same expression as K3's epilogue)
        RC(fan(c, [&](int i, pgh_ctx* k) -> int {
            return pgh_secagg_decode_device(k, base, prec, (const int64_t*)g->d_rs[(size_t)i], S,
                                            (float*)pgh_int::vec(k, pgh_int::V_DEC), pgh_int::stream_of(k));
        }, n));
    } else {
        // 2'. peer copies: GPU i gathers slice i of every GPU's sums into rows of a staging block and
        //     K3 folds the rows (sum + decode in one pass)
        RC(sync_all(c, n));
        RC(grow(c, &g->d_stage, &g->stage_cap, L * 8));
        RC(fan(c, [&](int i, pgh_ctx* k) -> int {
            DevSel d(pgh_int::device_of(k));
            const hipStream_t s = pgh_int::stream_of(k);
            int64_t* st = (int64_t*)g->d_stage[(size_t)i];
            for (int r = 0; r < n; ++r) {
                pgh_ctx* kr = g->kids[(size_t)r];
                const int64_t* src = (const int64_t*)pgh_int::vec(kr, pgh_int::V_SUM) + (int64_t)i * S;
                if (hipMemcpyPeerAsync(st + (int64_t)r * S, pgh_int::device_of(k), src, pgh_int::device_of(kr),
                                       (size_t)S * 8, s) != hipSuccess)
                    return pgh_int::fail(k, PGH_E_HIP, "peer copy of share sums from gpu %d failed", r);
            }
            pgh::SecaggArgs a{};
            a.shares = st;
            a.map = pgh::single_block(S);
            a.n_rows = n;
            a.p = S;
            a.sum_out = (int64_t*)g->d_rs[(size_t)i];
            a.dec_out = (float*)pgh_int::vec(k, pgh_int::V_DEC);
            a.divisor = div;
            a.flags = pgh::FL_FIRST | pgh::FL_FINAL;
            a.variant = -1;
            if (pgh::launch_secagg(a, s) != hipSuccess) return pgh_int::fail(k, PGH_E_HIP, "slice reduction failed");
            return PGH_OK;
        }, n));
    }
    // 4. host slices
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        const int64_t a = (int64_t)i * S, m = std::max<int64_t>(0, std::min(S, len - a));
        if (m == 0) return pgh_sync(k);
        DevSel d(pgh_int::device_of(k));
        const hipStream_t s = pgh_int::stream_of(k);
        if (sum_out && hipMemcpyAsync(sum_out + a, g->d_rs[(size_t)i], (size_t)m * 8, hipMemcpyDeviceToHost, s) != hipSuccess)
            return pgh_int::fail(k, PGH_E_HIP, "share-sum download failed");
        if (dec_out && hipMemcpyAsync(dec_out + a, pgh_int::vec(k, pgh_int::V_DEC), (size_t)m * 4,
                                      hipMemcpyDeviceToHost, s) != hipSuccess)
            return pgh_int::fail(k, PGH_E_HIP, "decoded download failed");
        if (hipStreamSynchronize(s) != hipSuccess) return pgh_int::fail(k, PGH_E_HIP, "stream sync failed");
        return PGH_OK;
    }, n);
}

int owner_of(pgh_ctx* c, int client, int* kid, int* local) {
    pgh_group* g = G(c);
    if (client < 0 || client >= g->per * (int)g->kids.size())
        return fail(c, PGH_E_ARG, "client %d outside the group's capacity %d", client, g->per * (int)g->kids.size());
    *kid = client / g->per;
    *local = client - *kid * g->per;
    return PGH_OK;
}

void note_client(pgh_group* g, int kid, int local) {
    auto& seen = g->kid_seen[(size_t)kid];
    if ((size_t)local >= seen.size()) seen.resize((size_t)local + 1, 0);
    if (!seen[(size_t)local]) { seen[(size_t)local] = 1; g->kid_clients[(size_t)kid] += 1; }
}

}  // namespace

extern "C" {

int pgh_create_group(int n_gpus, const int* devices, size_t pinned_bytes, pgh_ctx** out) {
    if (!out) return fail(nullptr, PGH_E_ARG, "out is NULL");
    *out = nullptr;
    if (n_gpus < 1 || n_gpus > 64) return fail(nullptr, PGH_E_ARG, "n_gpus %d outside [1,64]", n_gpus);
    auto* g = new pgh_group();
    for (int i = 0; i < n_gpus; ++i) g->devs.push_back(devices ? devices[i] : i);
    const int threads = std::max(2, std::min(16, pgh_int::usable_cpus() / n_gpus));
    for (int i = 0; i < n_gpus; ++i) {
        pgh_ctx* k = nullptr;
        const int rc = pgh_create(g->devs[(size_t)i], pinned_bytes, &k);
        if (rc) {
            const std::string why = pgh_last_error(nullptr);
            for (auto* kk : g->kids) pgh_destroy(kk);
            delete g;
            return fail(nullptr, rc, "group gpu %d (device %d): %s", i, devices ? devices[i] : i, why.c_str());
        }
        if (!std::getenv("PGH_COPY_THREADS")) (void)pgh_int::set_copy_threads(k, threads);
        g->kids.push_back(k);
    }
    g->fan.reset(new Fanout(n_gpus));
    g->kid_clients.assign((size_t)n_gpus, 0);
    g->kid_seen.assign((size_t)n_gpus, {});
    *out = pgh_int::new_group_ctx(g, g->devs[0]);
    return PGH_OK;
}

int pgh_group_size(const pgh_ctx* c, int* n) {
    if (!c || !n) return PGH_E_ARG;
    const pgh_group* g = pgh_int::group_of(c);
    *n = g ? (int)g->kids.size() : 1;
    return PGH_OK;
}

int pgh_group_child(pgh_ctx* c, int i, pgh_ctx** child) {
    if (!c || !child) return PGH_E_ARG;
    pgh_group* g = G(c);
    if (!g) {
        if (i != 0) return fail(c, PGH_E_ARG, "a single-GPU context has only child 0");
        *child = c;
        return PGH_OK;
    }
    if (i < 0 || i >= (int)g->kids.size()) return fail(c, PGH_E_ARG, "child %d outside [0,%zu)", i, g->kids.size());
    *child = g->kids[(size_t)i];
    return PGH_OK;
}

int pgh_set_client_sharding(pgh_ctx* c, int on) {
    if (!c) return PGH_E_ARG;
    pgh_group* g = G(c);
    if (!g) return on ? fail(c, PGH_E_UNSUPPORTED, "client sharding needs a group context") : PGH_OK;
    g->want_client_shard = on != 0;
    return PGH_OK;
}

int pgh_group_backend(pgh_ctx* c, int* rccl) {
    if (!c || !rccl) return PGH_E_ARG;
    pgh_group* g = G(c);
    *rccl = g ? g->backend : -1;
    return PGH_OK;
}

int pgh_group_allgather_resident(pgh_ctx* c, void** d_full_out) {
    if (!c) return PGH_E_ARG;
    pgh_group* g = G(c);
    if (!g) return fail(c, PGH_E_UNSUPPORTED, "pgh_group_allgather_resident needs a group context");
    RC(need_slab(c));
    if (g->client_shard || g->dtype != PGH_F32) return fail(c, PGH_E_STATE, "the resident checkpoint needs an fp32 param-sharded slab");
    const int n = g->active;
    const int64_t S = g->S;
    RC(ensure_backend(c, n));
    RC(grow(c, &g->d_full, &g->full_cap, (int64_t)n * S * 4));
    if (g->backend == 1) {
        g->rccl->group_start();
        for (int i = 0; i < n; ++i) {
            pgh_ctx* k = g->kids[(size_t)i];
            DevSel d(pgh_int::device_of(k));
            const ncclResult_t e = g->rccl->all_gather(pgh_int::vec(k, pgh_int::V_CKPT), g->d_full[(size_t)i], (size_t)S,
                                                       ncclFloat32, g->comms[(size_t)i], pgh_int::stream_of(k));
            if (e != ncclSuccess) {
                g->rccl->group_end();
                return fail(c, PGH_E_HIP, "ncclAllGather on gpu %d failed: %s", i, g->rccl->error_string(e));
            }
        }
        const ncclResult_t e = g->rccl->group_end();
        if (e != ncclSuccess) return fail(c, PGH_E_HIP, "ncclGroupEnd failed: %s", g->rccl->error_string(e));
    } else {
        RC(sync_all(c, n));
        RC(fan(c, [&](int i, pgh_ctx* k) -> int {
            DevSel d(pgh_int::device_of(k));
            for (int r = 0; r < n; ++r) {
                pgh_ctx* kr = g->kids[(size_t)r];
                if (hipMemcpyPeerAsync((float*)g->d_full[(size_t)i] + (int64_t)r * S, pgh_int::device_of(k),
                                       pgh_int::vec(kr, pgh_int::V_CKPT), pgh_int::device_of(kr), (size_t)S * 4,
                                       pgh_int::stream_of(k)) != hipSuccess)
                    return pgh_int::fail(k, PGH_E_HIP, "peer copy of the checkpoint shard of gpu %d failed", r);
            }
            return PGH_OK;
        }, n));
    }
    RC(sync_all(c, n));
    if (d_full_out)
        for (int i = 0; i < (int)g->kids.size(); ++i) d_full_out[i] = i < n ? g->d_full[(size_t)i] : nullptr;
    return PGH_OK;
}

}  // extern "C"

// ---- the public entry points on a group context (dispatched from pgh_*.cpp) ---------------------

namespace pgh_group_api {

void destroy(pgh_ctx* c) {
    pgh_group* g = G(c);
    for (size_t i = 0; i < g->kids.size(); ++i) (void)pgh_sync(g->kids[i]);
    if (g->rccl)
        for (auto cm : g->comms) g->rccl->comm_destroy(cm);
    free_exchange(g);
    g->fan.reset();
    for (auto* k : g->kids) pgh_destroy(k);
    delete g;
    pgh_int::free_group_ctx(c);
}

int set_layout(pgh_ctx* c, int n_tensors, const int64_t* numel) {
    pgh_group* g = G(c);
    if (n_tensors <= 0 || !numel) return fail(c, PGH_E_ARG, "need at least one tensor");
    int64_t P = 0;
    for (int k = 0; k < n_tensors; ++k) {
        if (numel[k] < 0) return fail(c, PGH_E_ARG, "tensor %d has negative numel", k);
        P += numel[k];
    }
    if (P <= 0) return fail(c, PGH_E_ARG, "model has no parameters");
    g->layout = false;
    g->max_clients = 0;
    g->client_shard = false;
    RC(fan(c, [&](int, pgh_ctx* k) -> int { return pgh_set_layout(k, n_tensors, numel); }, (int)g->kids.size()));
    g->numel.assign(numel, numel + n_tensors);
    g->P = P;
    g->lo = 0;
    g->hi = P;
    g->layout = true;
    return apply_shards(c, false);
}

int set_shard(pgh_ctx* c, int64_t lo, int64_t hi) {
    pgh_group* g = G(c);
    RC(need_layout(c));
    if (lo < 0 || hi > g->P || lo >= hi)
        return fail(c, PGH_E_ARG, "shard [%lld,%lld) outside [0,%lld)", (long long)lo, (long long)hi, (long long)g->P);
    g->lo = lo;
    g->hi = hi;
    g->max_clients = 0;
    g->client_shard = false;
    return apply_shards(c, false);
}

int reserve(pgh_ctx* c, int max_clients, int dtype, int n_parties) {
    pgh_group* g = G(c);
    RC(need_layout(c));
    if (max_clients <= 0) return fail(c, PGH_E_ARG, "max_clients must be positive");
    if (dtype != PGH_F32 && dtype != PGH_I64) return fail(c, PGH_E_ARG, "unknown dtype %d", dtype);
    const bool cs = g->want_client_shard && dtype == PGH_I64;
    g->max_clients = 0;
    RC(apply_shards(c, cs));
    const int n = (int)g->kids.size();
    g->client_shard = cs;
    g->per = cs ? (max_clients + n - 1) / n : max_clients;
    RC(fan(c, [&](int i, pgh_ctx* k) -> int {
        if (cs) RC(pgh_int::set_client_base(k, (int64_t)i * g->per));
        return pgh_reserve(k, g->per, dtype, n_parties);
    }, cs ? n : g->active));
    g->dtype = dtype;
    g->parties = dtype == PGH_F32 ? 1 : n_parties;
    g->max_clients = max_clients;
    g->kid_clients.assign((size_t)n, 0);
    g->kid_seen.assign((size_t)n, {});
    return PGH_OK;
}

int reset(pgh_ctx* c) {
    pgh_group* g = G(c);
    g->kid_clients.assign(g->kids.size(), 0);
    g->kid_seen.assign(g->kids.size(), {});
    if (!g->layout) return PGH_OK;
    return fan(c, [](int, pgh_ctx* k) -> int { return pgh_reset(k); }, g->client_shard ? (int)g->kids.size() : g->active);
}

int ingest_raw(pgh_ctx* c, int client, const void* flat, size_t nbytes, int dtype) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (!flat) return fail(c, PGH_E_ARG, "flat is NULL");
    const size_t es = dtype == PGH_F32 ? 4 : 8;
    if (g->client_shard) {
        int kid = 0, local = 0;
        RC(owner_of(c, client, &kid, &local));
        pgh_ctx* k = g->kids[(size_t)kid];
        const int rc = pgh_ingest_raw(k, local, flat, nbytes, dtype);
        if (rc) return fail(c, rc, "gpu %d: %s", kid, pgh_last_error(k));
        note_client(g, kid, local);
        return PGH_OK;
    }
    const size_t whole = (size_t)g->P * es * (size_t)g->parties, shard = (size_t)(g->hi - g->lo) * es * (size_t)g->parties;
    if (nbytes != whole && nbytes != shard)
        return fail(c, PGH_E_ARG, "client %d: got %zu bytes, layout needs %zu (model) or %zu (group range)", client,
                    nbytes, whole, shard);
    if (nbytes == whole) return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_ingest_raw(k, client, flat, nbytes, dtype); });
    if (g->parties != 1)
        return fail(c, PGH_E_ARG, "multi-party shares of a sub-range: pass the whole model's shares");
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        const uint8_t* src = (const uint8_t*)flat + (size_t)(kid_lo(g, i) - g->lo) * es;
        return pgh_ingest_raw(k, client, src, (size_t)(kid_hi(g, i) - kid_lo(g, i)) * es, dtype);
    });
}

int ingest_state(pgh_ctx* c, int client, const uint8_t* pb, size_t n) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (g->client_shard) return fail(c, PGH_E_STATE, "fp32 State diffs need a param-sharded slab");
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_ingest_state(k, client, pb, n); });
}

int ingest_state_shares(pgh_ctx* c, int client, int n_parties, const uint8_t* const* pbs, const size_t* ns) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (g->client_shard) {
        int kid = 0, local = 0;
        RC(owner_of(c, client, &kid, &local));
        pgh_ctx* k = g->kids[(size_t)kid];
        const int rc = pgh_ingest_state_shares(k, local, n_parties, pbs, ns);
        if (rc) return fail(c, rc, "gpu %d: %s", kid, pgh_last_error(k));
        note_client(g, kid, local);
        return PGH_OK;
    }
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_ingest_state_shares(k, client, n_parties, pbs, ns); });
}

int synth_ingest(pgh_ctx* c, uint64_t seed, int client0, int n) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (n <= 0 || client0 < 0) return fail(c, PGH_E_ARG, "bad client range %d + %d", client0, n);
    if (!g->client_shard) return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_synth_ingest(k, seed, client0, n); });
    const int nk = (int)g->kids.size();
    if ((int64_t)client0 + n > (int64_t)g->per * nk) return fail(c, PGH_E_ARG, "clients beyond the group's capacity");
    RC(fan(c, [&](int i, pgh_ctx* k) -> int {
        const int a = std::max(client0, i * g->per), b = std::min(client0 + n, (i + 1) * g->per);
        return a < b ? pgh_synth_ingest(k, seed, a - i * g->per, b - a) : PGH_OK;
    }, nk));
    for (int cl = client0; cl < client0 + n; ++cl) note_client(g, cl / g->per, cl % g->per);
    return PGH_OK;
}

int synth_fill(pgh_ctx* c, uint64_t seed, int n_clients) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (n_clients <= 0 || n_clients > g->max_clients)
        return fail(c, PGH_E_ARG, "n_clients %d outside (0,%d]", n_clients, g->max_clients);
    RC(reset(c));
    return synth_ingest(c, seed, 0, n_clients);
}

int set_synth_kind(pgh_ctx* c, int kind) {
    if (kind != 0 && kind != 1) return fail(c, PGH_E_ARG, "synthetic generator kind %d is not 0 or 1", kind);
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_set_synth_kind(k, kind); }, (int)G(c)->kids.size());
}

int set_ingest_ranges(pgh_ctx* c, int on) {
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_set_ingest_ranges(k, on); }, (int)G(c)->kids.size());
}

int set_weights(pgh_ctx* c, const float* w, int n) {
    if (!w || n <= 0) return fail(c, PGH_E_ARG, "need a non-empty weight vector");
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_set_weights(k, w, n); });
}

int fedavg(pgh_ctx* c, int mode, const float* ckpt, float* out) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (!ckpt || !out) return fail(c, PGH_E_ARG, "ckpt / out is NULL");
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        const int64_t off = kid_lo(g, i) - g->lo;
        return pgh_fedavg(k, mode, ckpt + off, out + off);
    });
}

int ckpt_upload(pgh_ctx* c, const float* ckpt, size_t nbytes) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (!ckpt) return fail(c, PGH_E_ARG, "ckpt is NULL");
    const size_t whole = 4 * (size_t)g->P, range = 4 * (size_t)(g->hi - g->lo);
    if (nbytes != whole && nbytes != range)
        return fail(c, PGH_E_ARG, "checkpoint: got %zu bytes, layout needs %zu (model) or %zu (group range)", nbytes,
                    whole, range);
    if (nbytes == whole) return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_ckpt_upload(k, ckpt, nbytes); });
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        return pgh_ckpt_upload(k, ckpt + (kid_lo(g, i) - g->lo), 4 * (size_t)(kid_hi(g, i) - kid_lo(g, i)));
    });
}

int ckpt_upload_state(pgh_ctx* c, const uint8_t* pb, size_t n) {
    RC(need_slab(c));
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_ckpt_upload_state(k, pb, n); });
}

int fedavg_resident(pgh_ctx* c, int mode) {
    RC(need_slab(c));
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_fedavg_resident(k, mode); });
}

int ckpt_download(pgh_ctx* c, float* out) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (!out) return fail(c, PGH_E_ARG, "out is NULL");
    return fan(c, [&](int i, pgh_ctx* k) -> int { return pgh_ckpt_download(k, out + (kid_lo(g, i) - g->lo)); });
}

int ckpt_patch_state(pgh_ctx* c, const uint8_t* tmpl, size_t n, uint8_t* out) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (!tmpl || !out) return fail(c, PGH_E_ARG, "tmpl / out is NULL");
    if (out != tmpl) {
        // the framing (everything outside the group range's payload slices) once, on this thread
        std::vector<pgh_state::Span> spans;
        std::string msg;
        const int rc = pgh_state::scan(tmpl, n, &spans, &msg);
        if (rc) return fail(c, rc, "checkpoint template State: %s", msg.c_str());
        size_t pos = 0;
        int64_t off = 0;
        for (auto& sp : spans) {
            const int64_t a = std::max(off, g->lo), b = std::min(off + sp.count, g->hi);
            if (a < b) {
                const size_t s0 = sp.offset + 4 * (size_t)(a - off), s1 = sp.offset + 4 * (size_t)(b - off);
                if (s0 < pos) { std::memcpy(out, tmpl, n); pos = n; break; }  // never from the walker
                std::memcpy(out + pos, tmpl + pos, s0 - pos);
                pos = s1;
            }
            off += sp.count;
        }
        if (n > pos) std::memcpy(out + pos, tmpl + pos, n - pos);
    }
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_int::patch_payloads(k, tmpl, n, out); });
}

int fold_slots(pgh_ctx* c, int mode, const int32_t* slots, int n, bool finish) {
    RC(need_slab(c));
    return fan(c, [&](int, pgh_ctx* k) -> int {
        return finish ? pgh_fold_slots_finish_resident(k, mode, slots, n) : pgh_fold_slots(k, mode, slots, n);
    });
}

int fold_restart(pgh_ctx* c) {
    RC(need_slab(c));
    return fan(c, [](int, pgh_ctx* k) -> int { return pgh_fold_slots_restart(k); });
}

int secagg(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (g->client_shard) return secagg_client_sharded(c, base, prec, sum_out, dec_out);
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        const int64_t off = kid_lo(g, i) - g->lo;
        return pgh_secagg(k, base, prec, sum_out ? sum_out + off : nullptr, dec_out ? dec_out + off : nullptr);
    });
}

int stream_begin(pgh_ctx* c, int kind, int fold_batch) {
    RC(need_slab(c));
    if (G(c)->client_shard) return fail(c, PGH_E_UNSUPPORTED, "STREAM use needs a param-sharded slab");
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_stream_begin(k, kind, fold_batch); });
}

int stream_flush(pgh_ctx* c) {
    RC(need_slab(c));
    return fan(c, [](int, pgh_ctx* k) -> int { return pgh_stream_flush(k); });
}

int stream_finish(pgh_ctx* c, const float* ckpt, float* out) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    if (!ckpt || !out) return fail(c, PGH_E_ARG, "ckpt / out is NULL");
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        const int64_t off = kid_lo(g, i) - g->lo;
        return pgh_stream_finish(k, ckpt + off, out + off);
    });
}

int stream_finish_resident(pgh_ctx* c) {
    RC(need_slab(c));
    return fan(c, [](int, pgh_ctx* k) -> int { return pgh_stream_finish_resident(k); });
}

int stream_finish_secagg(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out) {
    pgh_group* g = G(c);
    RC(need_slab(c));
    return fan(c, [&](int i, pgh_ctx* k) -> int {
        const int64_t off = kid_lo(g, i) - g->lo;
        return pgh_stream_finish_secagg(k, base, prec, sum_out ? sum_out + off : nullptr,
                                        dec_out ? dec_out + off : nullptr);
    });
}

int set_variant(pgh_ctx* c, int variant) {
    if (variant < -1 || variant > 23) return fail(c, PGH_E_ARG, "variant %d outside [-1,23]", variant);
    return fan(c, [&](int, pgh_ctx* k) -> int { return pgh_set_variant(k, variant); }, (int)G(c)->kids.size());
}

int effective_variant(pgh_ctx* c, int mode) {
    RC(need_layout(c));
    const int v = pgh_effective_variant(G(c)->kids[0], mode);
    if (v < 0) return fail(c, v, "gpu 0: %s", pgh_last_error(G(c)->kids[0]));
    return v;
}

// Sums of bytes and counts; times as the slowest GPU's (the GPUs run concurrently).
int stats(pgh_ctx* c, pgh_stats_t* out) {
    pgh_group* g = G(c);
    if (!out) return PGH_E_ARG;
    const int n = (int)g->kids.size();
    std::vector<pgh_stats_t> st((size_t)n);
    RC(fan(c, [&](int i, pgh_ctx* k) -> int { return pgh_stats(k, &st[(size_t)i]); }, n));
    pgh_stats_t r{};
    const int used = g->client_shard ? n : std::max(1, g->active);
    for (int i = 0; i < used; ++i) {
        const auto& s = st[(size_t)i];
        r.kernel_ms_last = std::max(r.kernel_ms_last, s.kernel_ms_last);
        r.kernel_ms_total = std::max(r.kernel_ms_total, s.kernel_ms_total);
        r.kernel_launches = std::max(r.kernel_launches, s.kernel_launches);
        r.kernel_bytes_last += s.kernel_bytes_last;
        r.kernel_bytes_total += s.kernel_bytes_total;
        r.h2d_ms_total = std::max(r.h2d_ms_total, s.h2d_ms_total);
        r.h2d_bytes_total += s.h2d_bytes_total;
        r.h2d_staged_bytes_total += s.h2d_staged_bytes_total;
        r.d2h_bytes_total += s.d2h_bytes_total;
        r.d2h_kernel_bytes_total += s.d2h_kernel_bytes_total;
        r.close_ms_last = std::max(r.close_ms_last, s.close_ms_last);
        r.ld = std::max(r.ld, s.ld);
        r.n_folded = std::max(r.n_folded, s.n_folded);
        r.kernel_busy_ms_total = std::max(r.kernel_busy_ms_total, s.kernel_busy_ms_total);
        if (g->client_shard) {
            r.n_clients += s.n_clients;
            r.max_clients += s.max_clients;
        } else {
            r.n_clients = std::max(r.n_clients, s.n_clients);
            r.max_clients = std::max(r.max_clients, s.max_clients);
        }
    }
    r.p_shard = g->hi - g->lo;
    *out = r;
    return PGH_OK;
}

int reset_stats(pgh_ctx* c) {
    return fan(c, [](int, pgh_ctx* k) -> int { return pgh_reset_stats(k); }, (int)G(c)->kids.size());
}

int sync(pgh_ctx* c) {
    return fan(c, [](int, pgh_ctx* k) -> int { return pgh_sync(k); }, (int)G(c)->kids.size());
}

}  // namespace pgh_group_api
