/* CPU oracle (scalar C restatement) -- TEST INFRASTRUCTURE ONLY.
 *
 * Loaded with ctypes by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
 * the checker; never linked into or called by the product library (pygrid_amd/).
 * Same semantics as oracle/oracle.py, written as plain scalar loops over a flat
 * [clients][ld] layout.  Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no -ffast-math:
 * x86-64 SSE float arithmetic is IEEE binary32 with denormals kept).
 *
 * Reference citations (under /root/reference):
 *   or_fedavg_mean      apps/node/src/app/main/model_centric/cycles/cycle_manager.py:276-296
 *   or_fedavg_iterative cycle_manager.py:266-269 + examples/model-centric/01-Create-plan.ipynb:450-454
 *   or_fedavg_weighted  build-owned (north_star "weighted FedAvg"; == mean at w == 1)
 *   or_secagg           PySyft 0.2.9 AdditiveSharingTensor/FixedPrecisionTensor as exercised by
 *                       tests/data_centric/test_basic_syft_operations.py:388-454
 */
#include <stdint.h>
#include <stddef.h>
#include <math.h>

#define GOLDEN 0x9E3779B97F4A7C15ull

static inline uint64_t sm64(uint64_t x) {
    uint64_t z = x + GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t or_row_key(uint64_t seed, uint64_t stream, uint64_t row) {
    uint64_t k = sm64(seed ^ (stream << 48));
    return sm64(k ^ (row * 0xD1B54A32D192ED03ull));
}

static inline float bits_to_f32(uint64_t b, float scale) {
    int64_t s = (int64_t)((b & 0xFFFF) + ((b >> 16) & 0xFFFF) + ((b >> 32) & 0xFFFF) + (b >> 48));
    volatile float v = (float)(s - 131070);  /* exact: |v| < 2^24 */
    return v * scale;
}

/* out[k] = synthetic value of (stream,row) at global param index idx0 + k, k < n */
void or_synth_f32(uint64_t seed, uint64_t stream, uint64_t row, int64_t idx0, int64_t n,
                  float scale, float* out) {
    uint64_t base = or_row_key(seed, stream, row);
    for (int64_t k = 0; k < n; ++k) out[k] = bits_to_f32(sm64(base + (uint64_t)(idx0 + k)), scale);
}

/* generator kind 1: one word per 4 params (global index g >> 2), u16 number g & 3, uniform */
void or_synth_f32_fast(uint64_t seed, uint64_t stream, uint64_t row, int64_t idx0, int64_t n,
                       float scale, float* out) {
    uint64_t base = or_row_key(seed, stream, row);
    const float s2 = 2.0f * scale;
    for (int64_t k = 0; k < n; ++k) {
        const uint64_t g = (uint64_t)(idx0 + k);
        const uint64_t h = sm64(base + (g >> 2));
        volatile float v = (float)((int32_t)((h >> (16 * (g & 3))) & 0xFFFF) - 32768);
        out[k] = v * s2;
    }
}

void or_synth_u64(uint64_t seed, uint64_t stream, uint64_t row, int64_t idx0, int64_t n,
                  uint64_t* out) {
    uint64_t base = or_row_key(seed, stream, row);
    for (int64_t k = 0; k < n; ++k) out[k] = sm64(base + (uint64_t)(idx0 + k));
}

/* cycle_manager.py:286 left fold from d0, :288 true division by float(N), :294 subtract. */
int or_fedavg_mean(const float* diffs, int n, int64_t ld, int64_t p, const float* ckpt, float* out) {
    if (n <= 0) return -1;
    const float fn = (float)n;
    for (int64_t i = 0; i < p; ++i) {
        float acc = diffs[i];
        for (int c = 1; c < n; ++c) acc = acc + diffs[(int64_t)c * ld + i];
        float avg = acc / fn;
        out[i] = ckpt[i] - avg;
    }
    return 0;
}

/* avg_plan: (avg * num + item) / (num + 1), three separately rounded ops per client. */
int or_fedavg_iterative(const float* diffs, int n, int64_t ld, int64_t p, const float* ckpt, float* out) {
    if (n <= 0) return -1;
    for (int64_t i = 0; i < p; ++i) {
        float a = diffs[i];
        for (int k = 1; k < n; ++k) {
            volatile float prod = a * (float)k;
            volatile float s = prod + diffs[(int64_t)k * ld + i];
            a = s / (float)(k + 1);
        }
        out[i] = ckpt[i] - a;
    }
    return 0;
}

float or_weight_total(const float* w, int n) {
    float t = w[0];
    for (int c = 1; c < n; ++c) t = t + w[c];
    return t;
}

int or_fedavg_weighted(const float* diffs, const float* w, int n, int64_t ld, int64_t p,
                       const float* ckpt, float* out) {
    if (n <= 0) return -1;
    const float wt = or_weight_total(w, n);
    for (int64_t i = 0; i < p; ++i) {
        volatile float acc = diffs[i] * w[0];
        for (int c = 1; c < n; ++c) {
            volatile float prod = diffs[(int64_t)c * ld + i] * w[c];
            acc = acc + prod;
        }
        out[i] = ckpt[i] - acc / wt;
    }
    return 0;
}

/* shares: [n][s][ld] int64.  Wrap sum (computed in uint64, which is the Z_2^64 ring),
 * decode = float32(int64) / float32(divisor).  sum_out and dec_out may be NULL. */
int or_secagg(const int64_t* shares, int n, int s, int64_t ld, int64_t p, float divisor,
              int64_t* sum_out, float* dec_out) {
    if (n <= 0 || s <= 0) return -1;
    for (int64_t i = 0; i < p; ++i) {
        uint64_t acc = 0;
        for (int c = 0; c < n; ++c)
            for (int q = 0; q < s; ++q) acc += (uint64_t)shares[((int64_t)c * s + q) * ld + i];
        if (sum_out) sum_out[i] = (int64_t)acc;
        if (dec_out) dec_out[i] = (float)(int64_t)acc / divisor;
    }
    return 0;
}
