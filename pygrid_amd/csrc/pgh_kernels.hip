// gfx950 (CDNA4, MI355X) kernels for the PyGrid cycle-close aggregation path.
//
// K1  k_fedavg<MODE_MEAN>      out = ckpt - (((d0 + d1) + d2) + ...) / N
//       restates cycle_manager.py:276-296 (reduce(th.add) -> th.div(., N) -> subtract)
//     k_fedavg<MODE_WEIGHTED>  out = ckpt - (sum_c w_c*d_c) / (sum_c w_c)   (build-owned)
// K2  k_fedavg<MODE_ITERATIVE> a = d0; a = (a*k + d_k)/(k+1); out = ckpt - a
//       restates cycle_manager.py:266-269 + 01-Create-plan.ipynb:450-454
// K3  k_secagg                 Z_2^64 wrap-sum over [clients*parties][P] int64 + fixed-point
//       decode float32(int64)/10^prec (PySyft 0.2.9 semantics)
//
// Design (DESIGN.md "Kernels"): every kernel is a single streaming pass over the slab held in
// HBM, column-blocked (SlabMap in pgh_kernels.h: blocks of ld columns, each block all rows,
// so a lane's walk down the client rows stays inside one compact block).  Parallelism is over
// the PARAMETER axis only: one lane owns a column (1 or 4 fp32, 1 or 2 int64) and walks the
// client rows in index order, so the fp32 fold order is exactly the reference's left fold
// (bit-exact, no tree/shuffle reordering).  U rows are issued before they are consumed to keep
// U loads per lane in flight.  No LDS: there is no reuse to stage, and no MFMA: this is a
// 0.25 flop/byte reduction, bound by HBM bandwidth.
//
// Build flags matter for parity: -ffp-contract=off (no a*k+d -> FMA), no fast-math, f32
// denormals kept, IEEE (correctly rounded) f32 division.
#include "pgh_kernels.h"

#include <algorithm>

namespace pgh {
namespace {

constexpr int BLOCK = 256;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t row_key(uint64_t seed, uint64_t stream, uint64_t row) {
    return sm64(sm64(seed ^ (stream << 48)) ^ (row * 0xD1B54A32D192ED03ull));
}

__device__ __forceinline__ float bits_to_f32(uint64_t b, float scale) {
    const uint32_t s = (uint32_t)(b & 0xFFFF) + (uint32_t)((b >> 16) & 0xFFFF) +
                       (uint32_t)((b >> 32) & 0xFFFF) + (uint32_t)(b >> 48);
    return (float)((int32_t)s - 131070) * scale;  // exact convert, one rounded multiply
}

template <bool NT>
__device__ __forceinline__ f32x4 ld4(const float* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    else return *reinterpret_cast<const f32x4*>(p);
}

template <bool NT>
__device__ __forceinline__ u64x2 ld2u(const int64_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(p));
    else return *reinterpret_cast<const u64x2*>(p);
}

// [p]-sized vectors (acc, ckpt, out) may end mid-column: the last column goes scalar.
__device__ __forceinline__ f32x4 ld4_tail(const float* base, int64_t q, int64_t p) {
    const int64_t i = 4 * q;
    if (i + 4 <= p) return *reinterpret_cast<const f32x4*>(base + i);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int e = 0; e < 4; ++e)
        if (i + e < p) v[e] = base[i + e];
    return v;
}

__device__ __forceinline__ void st4_tail(float* base, int64_t q, int64_t p, f32x4 v) {
    const int64_t i = 4 * q;
    if (i + 4 <= p) { *reinterpret_cast<f32x4*>(base + i) = v; return; }
    for (int e = 0; e < 4; ++e)
        if (i + e < p) base[i + e] = v[e];
}

// Lane element: VEC = 4 (one 16-byte column of 4 params, the default) or VEC = 1 (one param per
// lane: 4x the lanes, for shards too small to fill 256 CUs with 16-byte columns).
template <int VEC> struct Lane;
template <> struct Lane<4> {
    using T = f32x4;
    template <bool NT> static __device__ __forceinline__ T load(const float* p) { return ld4<NT>(p); }
    static __device__ __forceinline__ T load_tail(const float* b, int64_t q, int64_t p) { return ld4_tail(b, q, p); }
    static __device__ __forceinline__ void store_tail(float* b, int64_t q, int64_t p, T v) { st4_tail(b, q, p, v); }
};
template <> struct Lane<1> {
    using T = float;
    template <bool NT> static __device__ __forceinline__ T load(const float* p) {
        if constexpr (NT) return __builtin_nontemporal_load(p);
        else return *p;
    }
    static __device__ __forceinline__ T load_tail(const float* b, int64_t q, int64_t p) { return q < p ? b[q] : 0.f; }
    static __device__ __forceinline__ void store_tail(float* b, int64_t q, int64_t p, T v) { if (q < p) b[q] = v; }
};

template <int MODE, class T>
__device__ __forceinline__ T fold(T acc, T v, const float* w, int r) {
    if constexpr (MODE == MODE_MEAN) {
        return acc + v;                                   // th.add, cycle_manager.py:286
    } else {
        return acc + v * w[r];                            // MODE_WEIGHTED: product rounded, then add
    }
}

// Iterative plan step k (01-Create-plan.ipynb:453): t = avg * k + d (two roundings: no FMA under
// -ffp-contract=off), avg = t / (k + 1) with k and k + 1 promoted to f32 like th.tensor([k]).
// The IEEE division is replaced by (float)((double)t * rec), rec = RN_f64(1 / y), y = (float)(k+1):
// the double product is within ~2^-52 of t / y, which for a normal quotient is never an f32
// rounding midpoint and never within ~2^-49 of one, so the final rounding agrees bit for bit
// (tests/native/recip_div_check.c: 2e9 operand pairs against IEEE division).  A lane whose
// quotient could be below 2^-125 (0 < |t| < 2^-125 * y) sets `tiny`; the caller then redoes the
// batch with real divisions.  rec comes from a per-client table (scalar loads: k is uniform).
__device__ __forceinline__ float iter_step(float acc, float v, float kf, double rec, uint32_t thr, bool& tiny) {
    const float t = acc * kf + v;
    const uint32_t ut = __float_as_uint(t) & 0x7fffffffu;
    tiny |= (ut - 1u) < thr;  // thr = bits(2^-125 * y) - 1
    return (float)((double)t * rec);
}
__device__ __forceinline__ f32x4 iter_step(f32x4 acc, f32x4 v, float kf, double rec, uint32_t thr, bool& tiny) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = iter_step(acc[e], v[e], kf, rec, thr, tiny);
    return o;
}

// Slab row of the launch's row r: r itself (contiguous rows from a.diffs), or the r-th entry of
// the row table (IDX: report-time folds of scattered slots; the index is wave-uniform, so it is a
// scalar load from the kernarg segment).
template <bool IDX>
__device__ __forceinline__ size_t row_at(const RowTab* t, int r) {
    if constexpr (IDX) return (size_t)(uint32_t)t->rows[r];
    else return (size_t)r;
}

// Fold rows r .. r + nv - 1 (nv <= U, already loaded in v) into acc, in order.  nv is U for full
// batches (the guards fold away) and the wave-uniform remainder for the last one.
template <int MODE, int U, int W, class T>
__device__ __forceinline__ void fold_rows(T (&acc)[W], const T (&v)[U][W], const FedavgArgs& a, int r, int nv) {
    if constexpr (MODE != MODE_ITERATIVE) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < nv)
#pragma unroll
                for (int w = 0; w < W; ++w) acc[w] = fold<MODE>(acc[w], v[u][w], a.weights, r + u);
    } else {
        T acc0[W];
#pragma unroll
        for (int w = 0; w < W; ++w) acc0[w] = acc[w];
        bool tiny = false;
        const uint32_t k0 = (uint32_t)(a.client0 + r);  // client indices < 2^31
#pragma unroll
        for (int u0 = 0; u0 < U; u0 += 8) {
            double rec[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (u0 + j < U && u0 + j < nv) rec[j] = a.recips[r + u0 + j];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (u0 + j >= U || u0 + j >= nv) break;
                const uint32_t k = k0 + (uint32_t)(u0 + j);
                const float kf = (float)k, y = (float)(k + 1u);
                const uint32_t thr = __float_as_uint(0x1p-125f * y) - 1u;
#pragma unroll
                for (int w = 0; w < W; ++w) acc[w] = iter_step(acc[w], v[u0 + j][w], kf, rec[j], thr, tiny);
            }
        }
        if (tiny) {  // rare: a quotient near f32's subnormal range -- redo these rows dividing for real
#pragma unroll
            for (int w = 0; w < W; ++w) acc[w] = acc0[w];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u >= nv) break;
                const uint32_t k = k0 + (uint32_t)u;
                const float kf = (float)k, y = (float)(k + 1u);
#pragma unroll
                for (int w = 0; w < W; ++w) acc[w] = (acc[w] * kf + v[u][w]) / y;
            }
        }
    }
}

// W columns per lane (q0, q0 + qstep, ...: each load instruction of a wave still reads one
// contiguous span), all rows of the chunk, in order.  VEC consecutive params per column.
template <int MODE, int U, int W, bool NT, int VEC, bool IDX = false>
__device__ __forceinline__ void fedavg_columns(const FedavgArgs& a, const RowTab* tab, int64_t q0, int64_t qstep) {
    using L = Lane<VEC>;
    using T = typename L::T;
    const int n = a.n_rows;
    const int64_t ld = a.map.ld;
    const float* col[W];
#pragma unroll
    for (int w = 0; w < W; ++w) col[w] = a.diffs + a.map.at(VEC * (q0 + w * qstep));
    T acc[W];
    int r;
    if (a.flags & FL_FIRST) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            acc[w] = L::template load<NT>(col[w] + row_at<IDX>(tab, 0) * ld);  // fold starts at d0, not 0
            if constexpr (MODE == MODE_WEIGHTED) acc[w] = acc[w] * a.weights[0];
        }
        r = 1;
    } else {
#pragma unroll
        for (int w = 0; w < W; ++w) acc[w] = L::load_tail(a.acc_in, q0 + w * qstep, a.p);
        r = 0;
    }
    for (; r + U <= n; r += U) {
        T v[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int w = 0; w < W; ++w)
                v[u][w] = L::template load<NT>(col[w] + row_at<IDX>(tab, r + u) * ld);
        fold_rows<MODE, U, W>(acc, v, a, r, U);
    }
    if (r < n) {  // the last partial batch, its loads in flight together
        const int nv = n - r;
        T v[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < nv)
#pragma unroll
                for (int w = 0; w < W; ++w) v[u][w] = L::template load<NT>(col[w] + row_at<IDX>(tab, r + u) * ld);
        fold_rows<MODE, U, W>(acc, v, a, r, nv);
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const int64_t q = q0 + w * qstep;
        if (a.flags & FL_FINAL) {
            const T avg = (MODE == MODE_ITERATIVE) ? acc[w] : acc[w] / a.divisor;  // th.div, :288
            L::store_tail(a.out, q, a.p, L::load_tail(a.ckpt, q, a.p) - avg);     // :293-296
        } else {
            L::store_tail(a.acc, q, a.p, acc[w]);
        }
    }
}

// Software-pipelined column walk (variants 21/22): the loads of row batch i + 1 are issued before
// batch i is folded, so a lane keeps between U and 2U rows in flight instead of draining to zero
// between batches.  Two named buffers (no register copies that would wait on the new loads); the
// fold of one batch and the loads of the next sit in one basic block, so the wait counts only
// cover the batch being folded.  Same fold order as fedavg_columns: bit-identical.
template <int MODE, int U, bool NT, int VEC>
__device__ __forceinline__ void fedavg_columns_pipe(const FedavgArgs& a, int64_t q) {
    using L = Lane<VEC>;
    using T = typename L::T;
    const int n = a.n_rows;
    const int64_t ld = a.map.ld;
    const float* col = a.diffs + a.map.at(VEC * q);
    T acc[1];
    int r;
    if (a.flags & FL_FIRST) {
        acc[0] = L::template load<NT>(col);
        if constexpr (MODE == MODE_WEIGHTED) acc[0] = acc[0] * a.weights[0];
        r = 1;
    } else {
        acc[0] = L::load_tail(a.acc_in, q, a.p);
        r = 0;
    }
    T A[U][1], B[U][1];
    if (r + U <= n) {
#pragma unroll
        for (int u = 0; u < U; ++u) A[u][0] = L::template load<NT>(col + (size_t)(r + u) * ld);
        for (;;) {
            if (r + 2 * U <= n) {
#pragma unroll
                for (int u = 0; u < U; ++u) B[u][0] = L::template load<NT>(col + (size_t)(r + U + u) * ld);
                fold_rows<MODE, U, 1>(acc, A, a, r, U);
                r += U;
            } else {
                fold_rows<MODE, U, 1>(acc, A, a, r, U);
                r += U;
                break;
            }
            if (r + 2 * U <= n) {
#pragma unroll
                for (int u = 0; u < U; ++u) A[u][0] = L::template load<NT>(col + (size_t)(r + U + u) * ld);
                fold_rows<MODE, U, 1>(acc, B, a, r, U);
                r += U;
            } else {
                fold_rows<MODE, U, 1>(acc, B, a, r, U);
                r += U;
                break;
            }
        }
    }
    if (r < n) {  // the last partial batch, its loads in flight together
        const int nv = n - r;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < nv) A[u][0] = L::template load<NT>(col + (size_t)(r + u) * ld);
        fold_rows<MODE, U, 1>(acc, A, a, r, nv);
    }
    if (a.flags & FL_FINAL) {
        const T avg = (MODE == MODE_ITERATIVE) ? acc[0] : acc[0] / a.divisor;  // th.div, :288
        L::store_tail(a.out, q, a.p, L::load_tail(a.ckpt, q, a.p) - avg);     // :293-296
    } else {
        L::store_tail(a.acc, q, a.p, acc[0]);
    }
}

template <int MODE, int U, bool NT, int TB, int VEC>
__global__ __launch_bounds__(TB) void k_fedavg_pipe(FedavgArgs a, int64_t ncol) {
    for (int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x; q < ncol; q += (int64_t)gridDim.x * TB)
        fedavg_columns_pipe<MODE, U, NT, VEC>(a, q);
}

// Workgroup -> tile order.  Workgroups are dealt round robin over the 8 XCDs (wg % 8); XMAP gives
// each XCD a contiguous eighth of the tiles instead (A/B variant 23: does DRAM page locality
// across XCDs matter for a read-once stream?).
template <bool XMAP>
__device__ __forceinline__ int64_t tile_of_wg() {
    if constexpr (!XMAP) return blockIdx.x;
    const int64_t g = gridDim.x, per = g / 8, b = blockIdx.x;
    return b < per * 8 ? (b % 8) * per + b / 8 : b;
}

// Grid-stride over tiles of TB x W columns; a partial last tile goes one column per lane.
template <int MODE, int U, int W, bool NT, int TB, int VEC, bool IDX, bool XMAP = false>
__device__ __forceinline__ void fedavg_tiles(const FedavgArgs& a, const RowTab* tab, int64_t ncol) {
    const int64_t tile = (int64_t)TB * W;
    for (int64_t t0 = tile_of_wg<XMAP>() * tile; t0 < ncol; t0 += (int64_t)gridDim.x * tile) {
        const int64_t q0 = t0 + threadIdx.x;
        if (t0 + tile <= ncol) {
            fedavg_columns<MODE, U, W, NT, VEC, IDX>(a, tab, q0, TB);
        } else {
            for (int64_t q = q0; q < ncol && q < t0 + tile; q += TB)
                fedavg_columns<MODE, U, 1, NT, VEC, IDX>(a, tab, q, TB);
        }
    }
}

template <int MODE, int U, int W, bool NT, int TB, int VEC, bool XMAP = false>
__global__ __launch_bounds__(TB) void k_fedavg(FedavgArgs a, int64_t ncol) {
    fedavg_tiles<MODE, U, W, NT, TB, VEC, false, XMAP>(a, nullptr, ncol);
}

// The same fold over the slab rows listed in `tab` (report-time aggregation, pgh_fold_slots).
template <int MODE, int U, int W, bool NT, int TB, int VEC>
__global__ __launch_bounds__(TB) void k_fedavg_rows(FedavgArgs a, int64_t ncol, RowTab tab) {
    fedavg_tiles<MODE, U, W, NT, TB, VEC, true>(a, &tab, ncol);
}

// Z_2^64 lane element: VEC = 2 (16-byte column of 2 int64) or 1 (one int64 per lane).
template <int VEC> struct Lane64;
template <> struct Lane64<2> {
    using T = u64x2;
    template <bool NT> static __device__ __forceinline__ T load(const int64_t* p) { return ld2u<NT>(p); }
};
template <> struct Lane64<1> {
    using T = unsigned long long;
    template <bool NT> static __device__ __forceinline__ T load(const int64_t* p) {
        const T* q = reinterpret_cast<const T*>(p);
        if constexpr (NT) return __builtin_nontemporal_load(q);
        else return *q;
    }
};

template <int VEC>
__device__ __forceinline__ unsigned long long lane_elem(const typename Lane64<VEC>::T& v, int e) {
    if constexpr (VEC == 1) return v;
    else return v[e];
}

template <int VEC>
__device__ __forceinline__ void lane_set(typename Lane64<VEC>::T& v, int e, unsigned long long x) {
    if constexpr (VEC == 1) v = x;
    else v[e] = x;
}

template <int U, bool NT, int TB, int VEC>
__global__ __launch_bounds__(TB) void k_secagg(SecaggArgs a, int64_t ncol) {
    using L = Lane64<VEC>;
    using T = typename L::T;
    const int64_t stride = (int64_t)gridDim.x * TB;
    const int64_t ld = a.map.ld;
    for (int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x; q < ncol; q += stride) {
        const int64_t i = VEC * q;
        const int64_t* col = a.shares + a.map.at(i);
        const int ne = (int)(i + VEC <= a.p ? VEC : a.p - i);  // valid elements of this column
        T acc{};
        if (!(a.flags & FL_FIRST))
            for (int e = 0; e < ne; ++e) lane_set<VEC>(acc, e, a.acc[i + e]);
        int r = 0;
        for (; r + U <= a.n_rows; r += U) {
            T v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = L::template load<NT>(col + (size_t)(r + u) * ld);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u];  // wraps mod 2^64
        }
        if (r < a.n_rows) {  // last partial batch, its loads in flight together
            const int nv = a.n_rows - r;
            T v[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (u < nv) v[u] = L::template load<NT>(col + (size_t)(r + u) * ld);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (u < nv) acc += v[u];
        }
        for (int e = 0; e < ne; ++e) {
            const unsigned long long x = lane_elem<VEC>(acc, e);
            if (a.flags & FL_FINAL) {
                if (a.sum_out) a.sum_out[i + e] = (int64_t)x;
                if (a.dec_out) a.dec_out[i + e] = (float)(int64_t)x / a.divisor;  // float_prec decode
            } else {
                a.acc[i + e] = x;
            }
        }
    }
}

// Page-locked report ingest (pgh_ingest_state): one workgroup per chunk of a float payload that
// sits at an arbitrary byte offset of the DMA'd message.  After a head that brings the slab column
// to a multiple of 4, each lane moves 4 floats: one 16-byte load of the 4 dwords around them (plus
// the dword after, for an unaligned payload) funnel-shifted out (v_alignbyte), one 16-byte store
// into the blocked slab row (blocks are multiples of 64 columns, so 4 aligned columns never straddle
// one).  Bound by HBM like a copy: 4 B read + 4 B written per param, the message read once.
__global__ __launch_bounds__(BLOCK) void k_gather_f32(const uint8_t* bytes, const GChunk* tab, float* row,
                                                      SlabMap m) {
    const GChunk ch = tab[blockIdx.x];
    const int head = (int)min((int64_t)ch.n, (4 - (ch.dst & 3)) & 3);
    const int body = (ch.n - head) & ~3;
    const uint32_t sh = (uint32_t)(ch.src & 3);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(bytes + (ch.src & ~int64_t(3)));
    auto one = [&](int t) {
        const uint32_t lo = w[t];
        const uint32_t v = sh ? __builtin_amdgcn_alignbyte(w[t + 1], lo, sh) : lo;
        row[m.at(ch.dst + t)] = __uint_as_float(v);
    };
    if ((int)threadIdx.x < head) one((int)threadIdx.x);
    const int tail0 = head + body;
    if ((int)threadIdx.x < ch.n - tail0) one(tail0 + (int)threadIdx.x);
    for (int q = (int)threadIdx.x * 4; q < body; q += BLOCK * 4) {
        const int t = head + q;
        uint4 a;
        __builtin_memcpy(&a, w + t, 16);  // 4-byte aligned: a dwordx4 load (unaligned access is legal)
        float4 o;
        if (sh) {
            const uint32_t e = w[t + 4];
            o.x = __uint_as_float(__builtin_amdgcn_alignbyte(a.y, a.x, sh));
            o.y = __uint_as_float(__builtin_amdgcn_alignbyte(a.z, a.y, sh));
            o.z = __uint_as_float(__builtin_amdgcn_alignbyte(a.w, a.z, sh));
            o.w = __uint_as_float(__builtin_amdgcn_alignbyte(e, a.w, sh));
        } else {
            o = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
        }
        *reinterpret_cast<float4*>(row + m.at(ch.dst + t)) = o;
    }
}

// Decode of an already-summed Z_2^64 vector (client-sharded secagg: the per-rank share sums are
// reduce-scattered, then each rank decodes its param shard).  Same expression as k_secagg's
// FINAL epilogue, compiled with the same flags: bit-identical to the single-GPU decode.
__global__ __launch_bounds__(BLOCK) void k_secagg_decode(const int64_t* sum, float* dec, int64_t n, float divisor) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK)
        dec[i] = (float)sum[i] / divisor;
}

// KIND 0: one splitmix64 word per param -> Irwin-Hall(4 x u16).  KIND 1 ("fast", config 4's
// on-device data source): one word per 4 consecutive params (global index g >> 2), param g takes
// u16 number g & 3 of it, centred, times 2 * scale (same sigma ~ 1e-2): a quarter of the integer
// work, so the fill is bound by its HBM writes instead of the 64-bit multiplies (r01af).
// NT: non-temporal stores (the rows are read back by a fold only after the whole chunk is written:
// nothing to keep in L2 / MALL).
template <int KIND, bool NT>
__global__ __launch_bounds__(BLOCK) void k_synth_f32(float* out, SlabMap m, int64_t ncols, int n_rows, int64_t p,
                                                     uint64_t seed, uint64_t stream_id, int64_t row0, int64_t idx0,
                                                     float scale) {
    for (int64_t r = blockIdx.y; r < n_rows; r += gridDim.y) {
        const uint64_t key = row_key(seed, stream_id, (uint64_t)(row0 + r));
        float* row = out + (size_t)r * m.ld;
        for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < ncols / 4; q += (int64_t)gridDim.x * BLOCK) {
            f32x4 v;
            if constexpr (KIND == 0) {
                const uint64_t k0 = key + (uint64_t)(idx0 + 4 * q);
                if (4 * q + 4 <= p) {  // branch-free: four independent hash chains interleave
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = bits_to_f32(sm64(k0 + (uint64_t)e), scale);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[e] = (4 * q + e < p) ? bits_to_f32(sm64(k0 + (uint64_t)e), scale) : 0.f;
                }
            } else {
                const float s2 = 2.0f * scale;  // exact
                const int64_t g0 = idx0 + 4 * q;
                if ((g0 & 3) == 0) {  // the four params share one word
                    const uint64_t h = sm64(key + (uint64_t)(g0 >> 2));
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[e] = (4 * q + e < p) ? (float)((int32_t)((h >> (16 * e)) & 0xFFFF) - 32768) * s2 : 0.f;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int64_t g = g0 + e;
                        const uint64_t h = sm64(key + (uint64_t)(g >> 2));
                        v[e] = (4 * q + e < p) ? (float)((int32_t)((h >> (16 * (g & 3))) & 0xFFFF) - 32768) * s2 : 0.f;
                    }
                }
            }
            f32x4* dst = reinterpret_cast<f32x4*>(row + m.at(4 * q));  // 4 params never straddle a block
            if constexpr (NT) __builtin_nontemporal_store(v, dst);
            else *dst = v;
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_synth_shares(int64_t* out, SlabMap m, int64_t ncols, int n_parties,
                                                        int64_t p, uint64_t seed, int64_t client0, int64_t idx0,
                                                        float enc_scale) {
    const int64_t c = blockIdx.y;
    const uint64_t kx = row_key(seed, STREAM_SECRET, (uint64_t)(client0 + c));
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < ncols; i += (int64_t)gridDim.x * BLOCK) {
        int64_t* dst = out + (size_t)(c * n_parties) * m.ld + m.at(i);
        if (i >= p) {
            for (int s = 0; s < n_parties; ++s) dst[(size_t)s * m.ld] = 0;
            continue;
        }
        const uint64_t g = (uint64_t)(idx0 + i);
        const float x = bits_to_f32(sm64(kx + g), DIFF_SCALE);
        const float y = x * enc_scale;                  // fix_prec: x * base**prec in f32
        const uint64_t enc = (uint64_t)(int64_t)y;      // .long(): truncation toward zero
        uint64_t acc = 0;
        for (int s = 0; s < n_parties - 1; ++s) {
            const uint64_t sh = sm64(row_key(seed, STREAM_SHARE, (uint64_t)((client0 + c) * n_parties + s)) + g);
            dst[(size_t)s * m.ld] = (int64_t)sh;
            acc += sh;
        }
        dst[(size_t)(n_parties - 1) * m.ld] = (int64_t)(enc - acc);
    }
}

// Packed varints -> int64 (TensorData.contents_int64 of secagg share States): K4 below.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Inclusive prefix sum over a wave64 in DPP moves (row shifts inside each 16-lane row, then the
// row totals broadcast into the rows after them): no LDS round trips, unlike __shfl_up's
// ds_bpermute chain.
__device__ __forceinline__ int wave_inclusive_sum(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// The value whose bytes are win[s .. e] (s >= e - 9, win[-16 .. 1039] readable), from the 12 bytes
// at s (three funnel shifts of the four aligned dwords around it).  The 7-bit groups are summed
// whole bytes at a time in byte dot products: raw = sum_i b_i 128^i over bytes b_0 .. b_9, i.e.
// sum_i (v_i + 128 c_i) 128^i with v_i the 7-bit group and c_i the continuation bit.  c_i = 1 for
// every byte before the last (e), so raw = value + K(len) + (multiples of 2^(7 len) from the bytes
// past e), with K(len) = sum_{j=1}^{len-1} 2^(7j); subtracting K(10) differs from K(len) only by
// multiples of 2^(7 len) too, so value = (raw - K(10)) mod 2^(7 len) (all 64 bits at len 10).
__device__ __forceinline__ uint64_t varint_at(const uint8_t* win, int s, int e) {
    const uint32_t* wd = reinterpret_cast<const uint32_t*>(win + (s & ~3));
    const uint32_t d0 = wd[0], d1 = wd[1], d2 = wd[2], d3 = wd[3];
    const uint32_t sh = (uint32_t)(s & 3);
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);  // bytes 0-3 of the value
    const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);  // 4-7
    const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);  // 8-11
    constexpr uint32_t LO = 0x00008001u, HI = 0x80010000u;       // byte weights (1, 128, 0, 0), (0, 0, 1, 128)
    // b0 + 128 b1 + 2^14 (b2 + 128 b3) < 2^30: no wrap
    const uint32_t a = __builtin_amdgcn_udot4(w0, LO, 0u, false) + (__builtin_amdgcn_udot4(w0, HI, 0u, false) << 14);
    const uint32_t b = __builtin_amdgcn_udot4(w1, LO, 0u, false) + (__builtin_amdgcn_udot4(w1, HI, 0u, false) << 14);
    const uint32_t c = __builtin_amdgcn_udot4(w2, LO, 0u, false);  // b8 + 128 b9 (only b9's bit 0 stays, at 63)
    const uint64_t raw = (uint64_t)a + ((uint64_t)b << 28) + ((uint64_t)c << 56);
    constexpr uint64_t K10 = 0x8102040810204080ull;  // sum_{j=1}^{9} 2^(7j)
    const int cut = max(57 - __mul24(e - s, 7), 0);   // 64 - 7 len: the bits above the value (24-bit mul)
    return ((raw - K10) << cut) >> cut;
}

// Terminator bits of 16 bytes (bit k: byte k has bit 7 clear) in byte dot products: the 0x80 bytes
// of ~v & 0x80808080 weighted 1, 2, 4, 8 (16 .. 128 for the second dword) sum to 128 x the mask.
__device__ __forceinline__ uint32_t term_mask16(const u32x4& v) {
    const uint32_t t0 = ~v[0] & 0x80808080u, t1 = ~v[1] & 0x80808080u;
    const uint32_t t2 = ~v[2] & 0x80808080u, t3 = ~v[3] & 0x80808080u;
    const uint32_t m01 = __builtin_amdgcn_udot4(t0, 0x08040201u, __builtin_amdgcn_udot4(t1, 0x80402010u, 0u, false), false);
    const uint32_t m23 = __builtin_amdgcn_udot4(t2, 0x08040201u, __builtin_amdgcn_udot4(t3, 0x80402010u, 0u, false), false);
    return (m01 >> 7) | (m23 << 1);
}

// K4: one workgroup per chunk of <= VARINT_CHUNK bytes (16 KiB), one wave per 4 KiB of it.  Each
// wave loads its 4 KiB (four 1 KiB windows, 16 bytes per lane each) at once, counts the value ends
// (terminator bytes) in them, and the four counts -- one barrier -- give each wave its starting
// rank from the chunk's `first` (the host counts terminators per chunk while staging).  Then per
// window lane t decodes the values that END in its 16 bytes itself: a value is at most 10 bytes,
// so it starts in lane t's bytes or lane t - 1's, both staged in the wave's LDS window; its rank
// is a DPP wave prefix sum of the terminator counts, its start the last terminator of lane t - 1
// (DPP wave shift) or, for lane 0, the carry from the previous window (or the 16 bytes before the
// wave's 4 KiB).  The values leave through LDS by rank, in rows of 64 consecutive int64s.
// Rounds 2-5 ran a block form (a workgroup per 64 KiB chunk compacting the value ends of 4 KiB
// windows into an LDS list by rank, three barriers per window): 55.6-57.9 us per 111 MB message of
// shares against this form's 37.4-38.1 us (tools/exp_varint.cpp, profiles/r06m/, r06q/).
// Byte-level work on a stream PCIe fills at ~55 GB/s; HBM traffic is ~1.84 bytes per byte in.
constexpr int VWIN = 1024;                  // a window: 64 lanes x 16 bytes
constexpr int VSUB = 4096;                  // a wave's part of a chunk
constexpr int VNW = VSUB / VWIN;            // windows per wave
static_assert(VARINT_CHUNK == 4 * VSUB, "K4: four waves of VSUB bytes per chunk");
constexpr int VSTAGE = 256;  // values of a window staged per wave (int64 shares: <= 115 values of 9-10 bytes)
__global__ __launch_bounds__(256) void k_varint_decode(const uint8_t* bytes, const VChunk* chunks, int64_t* row,
                                                       SlabMap m, int64_t lo, int64_t hi) {
    __shared__ u32x4 lds[4][1 + 64 + 1];    // per wave: [0] the 16 bytes before the window, [65] slack
    __shared__ uint64_t stage[4][VSTAGE];    // per wave: the window's values by rank
    __shared__ int wcount[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32x4* const win4 = lds[wave];
    uint64_t* const stg = stage[wave];
    const uint8_t* const win = reinterpret_cast<const uint8_t*>(win4) + 16;  // win[-16 .. 1039]
    const VChunk ch = chunks[blockIdx.x];
    const int sub0 = wave * VSUB;                    // this wave's bytes: [sub0, sub0 + subn) of the chunk
    const int subn = max(0, min(VSUB, ch.n - sub0));  // (0 for the waves past a short chunk's end)
    const int p = 16 * lane;
    const u32x4 zero = {0, 0, 0, 0};
    // Loads are unconditional (a branch around a load makes hipcc wait for it at once): offsets past
    // the chunk clamp to its last 16 bytes, masked out by the byte counts; zero bytes before a
    // payload's start read as terminators (the first value starts at offset 0).
    const int last16 = (ch.n - 1) & ~15;
    const bool has_before = sub0 > 0 || ch.off > ch.span_off;
    const u32x4 b16 = *reinterpret_cast<const u32x4*>(bytes + ch.off + (has_before ? min(sub0, last16 + 16) - 16 : 0));
    u32x4 buf[VNW];
#pragma unroll
    for (int i = 0; i < VNW; ++i)
        buf[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(bytes + ch.off + min(sub0 + i * VWIN + p, last16)));
    // value ends per window (bit k: byte p + k ends a value), this wave's total, the waves before it
    uint32_t tms[VNW];
    int mine = 0;
#pragma unroll
    for (int i = 0; i < VNW; ++i) {
        uint32_t tm = term_mask16(buf[i]);
        const int lim = subn - i * VWIN - p;  // bytes of mine inside the wave's part
        if (lim < 16) tm &= lim > 0 ? (1u << lim) - 1u : 0u;
        tms[i] = tm;
        mine += __popc(tm);
    }
    const int wtot = __builtin_amdgcn_readlane(wave_inclusive_sum(mine), 63);
    if (lane == 0) wcount[wave] = wtot;
    __syncthreads();
    int64_t base = ch.first;
    for (int w = 0; w < wave; ++w) base += wcount[w];
    if (subn == 0) return;  // (after the barrier: every wave reaches it)
    const u32x4 before = has_before ? b16 : zero;
    const uint32_t tb = term_mask16(before);
    int carry = tb ? (31 - __clz(tb)) - 16 : -16;  // window offset of the last value end before the window
    if (lane == 0) win4[65] = zero;
    u32x4 last = before;  // lane 63: the previous window's last 16 bytes
#pragma unroll
    for (int i = 0; i < VNW; ++i) {
        if (i * VWIN >= subn) break;
        const u32x4 v = buf[i];
        const uint32_t tm = tms[i];
        win4[1 + lane] = v;
        if (lane == 63) win4[0] = last;
        const int cnt = __popc(tm);
        const int x = wave_inclusive_sum(cnt);
        const int total = __builtin_amdgcn_readlane(x, 63);
        // my last value end; lane t - 1's is where my first value starts (every full 16 bytes of
        // valid input hold a value end); lane 0 takes the carry
        const int mylast = tm ? p + 31 - __clz(tm) : -64;
        const int prev = __builtin_amdgcn_update_dpp(carry, mylast, 0x138, 0xf, 0xf, false);  // wave_shr:1
        const uint64_t with = __ballot(tm != 0);
        // the window's values inside the shard and in one slab block (the usual case): consecutive
        // addresses from one base
        const int64_t l0 = base - lo, l1 = base + total - 1 - lo;
        const bool flat = base >= lo && base + total <= hi && ((m.off + l0) >> m.bshift) == ((m.off + l1) >> m.bshift);
        int64_t* const dst0 = row + (flat ? m.at(l0) : 0);
        // LDS writes above, reads below: one wave, in order; keep the compiler from moving them
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int r = x - cnt, pe = prev;  // r: my first value's rank in the window
        uint32_t left = tm;
        auto next = [&]() -> uint64_t {  // my next value, in order (validated input: s >= e - 9)
            const int e = p + __ffs(left) - 1;
            const uint64_t val = varint_at(win, max(pe + 1, e - 9), e);
            pe = e;
            left &= left - 1;
            return val;
        };
        // wave-uniform branches: one loop per case rather than a branch per value (decoding a
        // lane's two values as two independent chains measured no faster, r06m)
        if (flat && total <= VSTAGE) {  // by rank into LDS, then out in rows of 64 consecutive values
            while (left) stg[r++] = next();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int q = lane; q < total; q += 64) dst0[q] = (int64_t)stg[q];
        } else if (flat) {  // a dense window (> VSTAGE values, short varints)
            while (left) dst0[r++] = (int64_t)next();
        } else {            // a shard or slab-block edge inside the window
            while (left) {
                const int64_t idx = base + r++;
                const uint64_t val = next();
                if (idx >= lo && idx < hi) row[m.at(idx - lo)] = (int64_t)val;
            }
        }
        if (with) carry = __builtin_amdgcn_readlane(mylast, 63 - __clzll(with));
        carry -= VWIN;
        base += total;
        last = v;
        // the next window's LDS writes come after this window's reads (in order within the wave)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

int cu_count() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}

// Variants (A/B in one process: tools/ab_variants.py; profiles/r01*/README.md).
//   id  loads  U (rows in flight)  W (cols/lane)  block  VEC (params/col)  grid
//   0   nt     8                   1              256    4                 one lane per column  <- big shards
//   1   nt     8                   1              256    4                 persistent, 4 blocks/CU
//   2   plain  8                   1              256    4                 one lane per column
//   3   plain  8                   1              256    4                 persistent
//   4   plain  16                  1              256    4                 one lane per column
//   5   plain  16                  1              256    4                 persistent
//   6   nt     16                  1              256    4                 one lane per column
//   7   nt     4                   2              256    4                 one lane per W columns
//   8   nt     8                   2              256    4                 one lane per W columns
//   9   nt     8                   1              512    4                 one lane per column
//   10  nt     4                   1              256    4                 one lane per column
//   11  nt     16                  1              64     4                 one lane per column
//   12  nt     16                  1              64     1                 one lane per param
//   13  nt     8                   1              256    1                 one lane per param
//   14  nt     32                  1              64     1                 one lane per param
//   15  nt     32                  1              64     4                 one lane per column
//   16  nt     48                  1              64     1                 one lane per param
//   17  nt     64                  1              64     1                 one lane per param
//   18  nt     32                  1              128    1                 one lane per param
//   19  nt     16                  1              512    4                 one lane per column
//   20  nt     8                   1              1024   4                 one lane per column
//   21  nt     8 (+8 next batch)   1              256    4                 one lane per column, pipelined
//   22  nt     4 (+4 next batch)   1              256    4                 one lane per column, pipelined
//   23  nt     8                   1              256    4                 as 0, each XCD a contiguous eighth
// nt loads won 2-5 % on the once-read diff stream (r01c).  Small shards are bound by lanes / CU
// balance, not by the loads: the auto choice (variant -1) picks by shard size and mode
// (auto_variant below, r01l measurements on the column-blocked slab).
constexpr int N_VARIANTS = 24;
constexpr int SECAGG_AUTO_VARIANT = 14;

inline unsigned grid_for(int64_t ncol, int64_t tile, bool persistent) {
    const int64_t full = (ncol + tile - 1) / tile;
    if (!persistent) return (unsigned)(full > 0 ? full : 1);
    const int64_t pers = (int64_t)cu_count() * 4;
    return (unsigned)(full < pers ? (full > 0 ? full : 1) : pers);
}

template <int MODE, int U, int W, bool NT, int TB, int VEC, bool XMAP = false>
hipError_t go_fedavg(const FedavgArgs& a, bool persistent, hipStream_t s) {
    const int64_t ncol = (a.p + VEC - 1) / VEC;
    k_fedavg<MODE, U, W, NT, TB, VEC, XMAP><<<grid_for(ncol, (int64_t)TB * W, persistent), TB, 0, s>>>(a, ncol);
    return hipGetLastError();
}

template <int MODE, int U, int W, bool NT, int TB, int VEC>
hipError_t go_fedavg_rows(const FedavgArgs& a, const RowTab& t, hipStream_t s) {
    const int64_t ncol = (a.p + VEC - 1) / VEC;
    k_fedavg_rows<MODE, U, W, NT, TB, VEC><<<grid_for(ncol, (int64_t)TB * W, false), TB, 0, s>>>(a, ncol, t);
    return hipGetLastError();
}

// Indexed folds exist for the shapes the auto choice picks (auto_variant); an explicitly chosen
// variant outside them runs the auto shape for its shard.
template <int MODE>
hipError_t dispatch_fedavg_rows(const FedavgArgs& a, const RowTab& t, int variant, hipStream_t s) {
    switch (variant) {
    case 11: return go_fedavg_rows<MODE, 16, 1, true, 64, 4>(a, t, s);
    case 14: return go_fedavg_rows<MODE, 32, 1, true, 64, 1>(a, t, s);
    case 17: return go_fedavg_rows<MODE, 64, 1, true, 64, 1>(a, t, s);
    default: return go_fedavg_rows<MODE, 8, 1, true, 256, 4>(a, t, s);  // variant 0
    }
}

template <int MODE, int U, int TB, int VEC>
hipError_t go_fedavg_pipe(const FedavgArgs& a, hipStream_t s) {
    const int64_t ncol = (a.p + VEC - 1) / VEC;
    k_fedavg_pipe<MODE, U, true, TB, VEC><<<grid_for(ncol, TB, false), TB, 0, s>>>(a, ncol);
    return hipGetLastError();
}

template <int MODE>
hipError_t dispatch_fedavg(const FedavgArgs& a, int variant, hipStream_t s) {
    switch (variant) {
    case 0: return go_fedavg<MODE, 8, 1, true, 256, 4>(a, false, s);
    case 1: return go_fedavg<MODE, 8, 1, true, 256, 4>(a, true, s);
    case 2: return go_fedavg<MODE, 8, 1, false, 256, 4>(a, false, s);
    case 3: return go_fedavg<MODE, 8, 1, false, 256, 4>(a, true, s);
    case 4: return go_fedavg<MODE, 16, 1, false, 256, 4>(a, false, s);
    case 5: return go_fedavg<MODE, 16, 1, false, 256, 4>(a, true, s);
    case 6: return go_fedavg<MODE, 16, 1, true, 256, 4>(a, false, s);
    case 7: return go_fedavg<MODE, 4, 2, true, 256, 4>(a, false, s);
    case 8: return go_fedavg<MODE, 8, 2, true, 256, 4>(a, false, s);
    case 9: return go_fedavg<MODE, 8, 1, true, 512, 4>(a, false, s);
    case 10: return go_fedavg<MODE, 4, 1, true, 256, 4>(a, false, s);
    case 11: return go_fedavg<MODE, 16, 1, true, 64, 4>(a, false, s);
    case 12: return go_fedavg<MODE, 16, 1, true, 64, 1>(a, false, s);
    case 13: return go_fedavg<MODE, 8, 1, true, 256, 1>(a, false, s);
    case 14: return go_fedavg<MODE, 32, 1, true, 64, 1>(a, false, s);
    case 15: return go_fedavg<MODE, 32, 1, true, 64, 4>(a, false, s);
    case 16: return go_fedavg<MODE, 48, 1, true, 64, 1>(a, false, s);
    case 17: return go_fedavg<MODE, 64, 1, true, 64, 1>(a, false, s);
    case 18: return go_fedavg<MODE, 32, 1, true, 128, 1>(a, false, s);
    case 19: return go_fedavg<MODE, 16, 1, true, 512, 4>(a, false, s);
    case 20: return go_fedavg<MODE, 8, 1, true, 1024, 4>(a, false, s);
    case 21: return go_fedavg_pipe<MODE, 8, 256, 4>(a, s);
    case 22: return go_fedavg_pipe<MODE, 4, 256, 4>(a, s);
    case 23: return go_fedavg<MODE, 8, 1, true, 256, 4, true>(a, false, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

// Measured on MI355X, column-blocked slab (r01l, tools/sweep_r01l.sh; GB/s of algorithmic bytes):
//   P = 11.69M x 1K:     mean v0 6930 / v6 6921 / v15 6882 / v11 6861 / v14 6576
//                        iterative v0 6845 / v6 6828 / v15 6817;  weighted v15 7035 / v0 6921
//   P = 3M x 1K:         mean v6 6829 / v0 6822 / v15 6773;  iterative v6 6619 / v0 6615
//   P = 1M x 3K:         mean v0 6921 / v6 6912 / v11 6769;  iterative v0 6753 / v6 6555
//   P = 311,650 x 10K:   mean v11 6885 / v15 6645 / v0 5753;  iterative v12 5711 / v14 5670 / v11 5351
//   P = 100K x 30K:      mean v11 6403 / v12 6251;  iterative v14 4742 / v12 4465 / v11 2784
//   single block (P < 65,536; layout unchanged from r01g): P = 50K x 60K v14 6088 / v12 4013
// Pipelined walk (r01w): P = 11.69M x 1K mean v0 6809 / v21 6798 / v22 6822, iterative 6834 / 6864 /
//   6834, weighted 6816 / 6831 / 6820; 1M x 3K and 12.5M x 1K within 0.4 %: not latency-bound.
// Iterative fold with the reciprocal-multiply division (r01o, tools/ab_iterative.sh):
//   P = 50K x 60K v17 3665 / v14 3496;  100K x 30K v14 5970 / v17 5616;  311,650 x 10K v11 6359 /
//   v14 5894;  1M x 3K v0 6755;  11.69M x 1K v0 6846  (IEEE division: 3209 / 4757 / 5784 / 6753 / 6845)
// Big shards: 16-byte columns in 256-thread blocks (the blocked slab made them 5 % faster than one
// param per lane).  Below ~786K params those give < 768 workgroups for 256 CUs, so 64-thread
// blocks (CU balance); below ~200K params one param per lane (lanes), with deeper row pipelines
// for the iterative fold of the smallest shards (few waves: latency).
int auto_variant(int64_t p, int mode) {
    // under 80 K params (many clients per launch): the mean's 64-row walk (v17) up to ~45 K
    // (+10-37 % over v14 at 10-40 K x 3,000), the iterative fold's 32-row walk in 128-thread blocks
    // (v18) from ~35 K (+7-29 % over v17 at 40-65 K; below that the division chain ties them all),
    // weighted unchanged, r02ax / r02ay
    if (p < 80000) {
        if (mode == MODE_ITERATIVE) return p < 35000 ? 17 : 18;
        return mode == MODE_MEAN && p < 45000 ? 17 : 14;
    }
    // 80-125 K: the weighted fold on one param per lane with 16 rows in flight (v12: +21 % at
    // 100 K x 3,000; at 150-190 K v11 matches or beats it, r02bc / r02bd)
    if (p < 200000) return mode == MODE_ITERATIVE ? 14 : mode == MODE_WEIGHTED && p < 125000 ? 12 : 11;
    // between 200 K and 786 K params: the iterative fold takes one param per lane in 256-thread
    // blocks up to ~360 K (v13: 5.9-6.6 TB/s vs v11's 4.5-5.4 at 200-311 K x 1,000) and the
    // 16-byte columns of v0 above (6.3-6.7 vs 6.1-6.5); the mean takes v13 up to ~360 K too
    // (6.5 vs 5.9 at 200 K, equal at 250-350 K); weighted stays on v11 (mixed), r02ar-r02au
    if (p < 786432) {
        if (mode == MODE_ITERATIVE) return p < 360000 ? 13 : 0;
        return mode == MODE_MEAN && p < 360000 ? 13 : 11;
    }
    return 0;  // r01p (masked last batch): mean 6918, iterative 6910, weighted 6905 (v15 6647)
}

template <int U, bool NT, int TB, int VEC>
hipError_t go_secagg(const SecaggArgs& a, hipStream_t s) {
    const int64_t ncol = (a.p + VEC - 1) / VEC;
    k_secagg<U, NT, TB, VEC><<<grid_for(ncol, TB, false), TB, 0, s>>>(a, ncol);
    return hipGetLastError();
}

// Geometry a kernel may rely on: rows 16-byte aligned (ld a multiple of 4), blocks
// power-of-two wide (or one block holding the launch's columns), the launch's first column
// 4-aligned so a 16-byte column never straddles a block.
bool valid_map(const SlabMap& m, int64_t p) {
    if (m.ld <= 0 || (m.ld & 3) || (m.off & 3) || m.off < 0) return false;
    if (m.bshift == 62) return m.bmask == (int64_t(1) << 62) - 1 && m.off + p <= m.ld;
    return m.bshift > 0 && m.bshift < 40 && (int64_t(1) << m.bshift) == m.ld && m.bmask == m.ld - 1 && m.bstride >= m.ld;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

hipError_t launch_fedavg(const FedavgArgs& a_, hipStream_t s) {
    FedavgArgs a = a_;
    if (!a.acc_in) a.acc_in = a.acc;
    if (!(a.flags & FL_FIRST) && (!a.acc_in || !aligned16(a.acc_in))) return hipErrorInvalidValue;
    if (a.p <= 0 || a.n_rows < 0 || !valid_map(a.map, a.p)) return hipErrorInvalidValue;
    if ((a.flags & FL_FIRST) && a.n_rows < 1) return hipErrorInvalidValue;
    if (a.n_rows > 0 && (!a.diffs || (reinterpret_cast<uintptr_t>(a.diffs) & 15))) return hipErrorInvalidValue;
    if (!(a.flags & FL_FIRST) && (!a.acc || (reinterpret_cast<uintptr_t>(a.acc) & 15))) return hipErrorInvalidValue;
    if (!(a.flags & FL_FINAL) && (!a.acc || (reinterpret_cast<uintptr_t>(a.acc) & 15))) return hipErrorInvalidValue;
    if ((a.flags & FL_FINAL) && (!a.ckpt || !a.out || (reinterpret_cast<uintptr_t>(a.ckpt) & 15) ||
                                 (reinterpret_cast<uintptr_t>(a.out) & 15)))
        return hipErrorInvalidValue;
    if (a.mode == MODE_WEIGHTED && a.n_rows > 0 && !a.weights) return hipErrorInvalidValue;
    if (a.mode == MODE_ITERATIVE && a.n_rows > 0 && !a.recips) return hipErrorInvalidValue;
    const int v = a.variant < 0 ? auto_variant(a.p, a.mode) : a.variant;
    switch (a.mode) {
    case MODE_MEAN: return dispatch_fedavg<MODE_MEAN>(a, v, s);
    case MODE_ITERATIVE: return dispatch_fedavg<MODE_ITERATIVE>(a, v, s);
    case MODE_WEIGHTED: return dispatch_fedavg<MODE_WEIGHTED>(a, v, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fedavg_rows(const FedavgArgs& a_, const RowTab& t, hipStream_t s) {
    FedavgArgs a = a_;
    if (!a.acc_in) a.acc_in = a.acc;
    if (!(a.flags & FL_FIRST) && (!a.acc_in || !aligned16(a.acc_in))) return hipErrorInvalidValue;
    if (a.n_rows > ROWTAB_MAX) return hipErrorInvalidValue;
    if (a.p <= 0 || a.n_rows < 0 || !valid_map(a.map, a.p)) return hipErrorInvalidValue;
    if ((a.flags & FL_FIRST) && a.n_rows < 1) return hipErrorInvalidValue;
    if (a.n_rows > 0 && (!a.diffs || (reinterpret_cast<uintptr_t>(a.diffs) & 15))) return hipErrorInvalidValue;
    if (!(a.flags & FL_FIRST) && (!a.acc || (reinterpret_cast<uintptr_t>(a.acc) & 15))) return hipErrorInvalidValue;
    if (!(a.flags & FL_FINAL) && (!a.acc || (reinterpret_cast<uintptr_t>(a.acc) & 15))) return hipErrorInvalidValue;
    if ((a.flags & FL_FINAL) && (!a.ckpt || !a.out || (reinterpret_cast<uintptr_t>(a.ckpt) & 15) ||
                                 (reinterpret_cast<uintptr_t>(a.out) & 15)))
        return hipErrorInvalidValue;
    if (a.mode == MODE_WEIGHTED && a.n_rows > 0 && !a.weights) return hipErrorInvalidValue;
    if (a.mode == MODE_ITERATIVE && a.n_rows > 0 && !a.recips) return hipErrorInvalidValue;
    int v = auto_variant(a.p, a.mode);
    if (a.variant == 0 || a.variant == 11 || a.variant == 14 || a.variant == 17) v = a.variant;
    switch (a.mode) {
    case MODE_MEAN: return dispatch_fedavg_rows<MODE_MEAN>(a, t, v, s);
    case MODE_ITERATIVE: return dispatch_fedavg_rows<MODE_ITERATIVE>(a, t, v, s);
    case MODE_WEIGHTED: return dispatch_fedavg_rows<MODE_WEIGHTED>(a, t, v, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_secagg(const SecaggArgs& a, hipStream_t s) {
    if (a.p <= 0 || a.n_rows < 0 || !valid_map(a.map, a.p)) return hipErrorInvalidValue;
    if (a.n_rows > 0 && (!a.shares || (reinterpret_cast<uintptr_t>(a.shares) & 15))) return hipErrorInvalidValue;
    if (!(a.flags & FL_FINAL) && !a.acc) return hipErrorInvalidValue;
    if (!(a.flags & FL_FIRST) && !a.acc) return hipErrorInvalidValue;
    // auto: one int64 per lane, 32 rows in flight, 64-thread blocks (r01l, blocked slab: 6878 GB/s
    // at ResNet-18 x 1,000 x 2 (v16 6886, 16-byte columns v0 6613), 6747 at 311,650 x 2,500 x 2)
    const int v = a.variant < 0 ? SECAGG_AUTO_VARIANT : a.variant;
    if (v >= N_VARIANTS) return hipErrorInvalidValue;
    switch (v) {  // same load policy / depth / block / lane width as the fedavg variant of that id
    case 1: case 3: case 5: {  // persistent grids
        const int64_t ncol = (a.p + 1) / 2;
        const unsigned g = grid_for(ncol, BLOCK, true);
        if (v == 1) k_secagg<8, true, BLOCK, 2><<<g, BLOCK, 0, s>>>(a, ncol);
        else if (v == 3) k_secagg<8, false, BLOCK, 2><<<g, BLOCK, 0, s>>>(a, ncol);
        else k_secagg<16, false, BLOCK, 2><<<g, BLOCK, 0, s>>>(a, ncol);
        return hipGetLastError();
    }
    case 2: return go_secagg<8, false, 256, 2>(a, s);
    case 4: return go_secagg<16, false, 256, 2>(a, s);
    case 6: return go_secagg<16, true, 256, 2>(a, s);
    case 7: case 10: return go_secagg<4, true, 256, 2>(a, s);
    case 11: return go_secagg<16, true, 64, 2>(a, s);
    case 12: return go_secagg<16, true, 64, 1>(a, s);
    case 13: return go_secagg<8, true, 256, 1>(a, s);
    case 14: return go_secagg<32, true, 64, 1>(a, s);
    case 15: return go_secagg<32, true, 64, 2>(a, s);
    case 16: return go_secagg<48, true, 64, 1>(a, s);
    case 17: return go_secagg<64, true, 64, 1>(a, s);
    case 18: return go_secagg<32, true, 128, 1>(a, s);
    default: return go_secagg<8, true, 256, 2>(a, s);
    }
}

hipError_t launch_synth_f32(float* out, const SlabMap& m, int64_t ncols, int n_rows, int64_t p, uint64_t seed,
                            uint64_t stream_id, int64_t row0, int64_t idx0, float scale, hipStream_t s,
                            int64_t max_wgs, int kind, bool nt) {
    if (!out || n_rows < 0 || n_rows > 65535 || ncols < p || (ncols & 3) || m.off != 0 || !valid_map(m, 0) ||
        (kind != 0 && kind != 1) ||
        (m.bshift == 62 && ncols > m.ld) || (reinterpret_cast<uintptr_t>(out) & 15))
        return hipErrorInvalidValue;
    if (n_rows == 0 || ncols == 0) return hipSuccess;
    int64_t gx = (ncols / 4 + BLOCK - 1) / BLOCK;
    if (gx > 1024) gx = 1024;
    int64_t gy = n_rows;
    if (max_wgs > 0) {  // bounded grid: rows strided, leaves CU slots to a fold running beside it
        if (gx > max_wgs) gx = max_wgs;
        gy = std::max<int64_t>(1, std::min<int64_t>(n_rows, max_wgs / gx));
    }
    const dim3 grid((unsigned)gx, (unsigned)gy);
    if (kind == 1 && nt)
        k_synth_f32<1, true><<<grid, BLOCK, 0, s>>>(out, m, ncols, n_rows, p, seed, stream_id, row0, idx0, scale);
    else if (kind == 1)
        k_synth_f32<1, false><<<grid, BLOCK, 0, s>>>(out, m, ncols, n_rows, p, seed, stream_id, row0, idx0, scale);
    else if (nt)
        k_synth_f32<0, true><<<grid, BLOCK, 0, s>>>(out, m, ncols, n_rows, p, seed, stream_id, row0, idx0, scale);
    else
        k_synth_f32<0, false><<<grid, BLOCK, 0, s>>>(out, m, ncols, n_rows, p, seed, stream_id, row0, idx0, scale);
    return hipGetLastError();
}

hipError_t launch_varint_decode(const uint8_t* bytes, const VChunk* chunks, int n_chunks, int64_t* row,
                                const SlabMap& m, int64_t lo, int64_t hi, hipStream_t s) {
    if (n_chunks < 0 || (n_chunks > 0 && (!bytes || !chunks || !row)) || (reinterpret_cast<uintptr_t>(bytes) & 15) ||
        m.off != 0 || !valid_map(m, 0) || lo > hi)
        return hipErrorInvalidValue;
    if (n_chunks == 0) return hipSuccess;
    k_varint_decode<<<(unsigned)n_chunks, 256, 0, s>>>(bytes, chunks, row, m, lo, hi);
    return hipGetLastError();
}

hipError_t launch_gather_f32(const uint8_t* bytes, const GChunk* chunks, int n_chunks, float* row, const SlabMap& m,
                             hipStream_t s) {
    // 16-byte row stores: the row and the map's column offset 4-aligned (blocks are multiples of 4)
    if (n_chunks < 0 || (n_chunks > 0 && (!bytes || !chunks || !row)) || (reinterpret_cast<uintptr_t>(bytes) & 3) ||
        (reinterpret_cast<uintptr_t>(row) & 15) || (m.off & 3) || (m.ld & 3) || (m.bstride & 3))
        return hipErrorInvalidValue;
    if (n_chunks == 0) return hipSuccess;
    k_gather_f32<<<(unsigned)n_chunks, BLOCK, 0, s>>>(bytes, chunks, row, m);
    return hipGetLastError();
}

hipError_t launch_secagg_decode(const int64_t* sum, float* dec, int64_t n, float divisor, hipStream_t s) {
    if (n < 0 || (n > 0 && (!sum || !dec))) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    int64_t g = (n + BLOCK - 1) / BLOCK;
    if (g > 8192) g = 8192;
    k_secagg_decode<<<(unsigned)g, BLOCK, 0, s>>>(sum, dec, n, divisor);
    return hipGetLastError();
}

hipError_t launch_synth_shares(int64_t* out, const SlabMap& m, int64_t ncols, int n_clients, int n_parties,
                               int64_t p, uint64_t seed, int64_t client0, int64_t idx0, float enc_scale,
                               hipStream_t s) {
    if (!out || n_clients < 0 || n_clients > 65535 || n_parties < 1 || ncols < p || m.off != 0 || !valid_map(m, 0) ||
        (m.bshift == 62 && ncols > m.ld))
        return hipErrorInvalidValue;
    if (n_clients == 0 || ncols == 0) return hipSuccess;
    int64_t gx = (ncols + BLOCK - 1) / BLOCK;
    if (gx > 1024) gx = 1024;
    k_synth_shares<<<dim3((unsigned)gx, (unsigned)n_clients), BLOCK, 0, s>>>(out, m, ncols, n_parties, p, seed,
                                                                            client0, idx0, enc_scale);
    return hipGetLastError();
}

}  // namespace pgh
