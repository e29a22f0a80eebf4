// Internal launcher interface between the C-ABI context code (pgh_api.cpp) and the gfx950
// kernels (pgh_kernels.hip).  Not installed; the public surface is include/pgh_api.h.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pgh {

// fedavg modes (same numbering as PGH_MEAN / PGH_ITERATIVE_MEAN / PGH_WEIGHTED_MEAN)
enum { MODE_MEAN = 0, MODE_ITERATIVE = 1, MODE_WEIGHTED = 2 };
// flags for a chunked (client-streaming) reduction
enum { FL_FIRST = 1, FL_FINAL = 2 };

struct FedavgArgs {
    const float* diffs;     // [n_rows][ld] fp32, rows = clients client0 .. client0+n_rows-1
    int64_t ld;             // row stride in elements, multiple of 4, >= p
    int n_rows;
    int64_t client0;        // global index of row 0 (iterative k, weight index)
    int64_t p;              // params in this shard
    const float* weights;   // [n_rows] device, MODE_WEIGHTED only
    float* acc;             // [p] running state; read unless FL_FIRST, written unless FL_FINAL
    const float* ckpt;      // [p], FL_FINAL only
    float* out;             // [p], FL_FINAL only
    float divisor;          // float(N) or sum of weights, FL_FINAL of MEAN / WEIGHTED
    int flags;
    int mode;
    int variant;            // kernel variant (table in pgh_kernels.hip); < 0 = auto by shard size
};
hipError_t launch_fedavg(const FedavgArgs& a, hipStream_t s);

struct SecaggArgs {
    const int64_t* shares;  // [n_rows][ld] int64 (rows = clients x parties), ld even, >= p
    int64_t ld;
    int n_rows;
    int64_t p;
    uint64_t* acc;          // [p] running wrap-sum; read unless FL_FIRST, written unless FL_FINAL
    int64_t* sum_out;       // [p] nullable, FL_FINAL only
    float* dec_out;         // [p] nullable, FL_FINAL only
    float divisor;          // float(base ** prec)
    int flags;
    int variant;
};
hipError_t launch_secagg(const SecaggArgs& a, hipStream_t s);
// The fp32 fold variant the auto choice (variant < 0) picks for a shard of p params.
int auto_variant(int64_t p, int mode);

// Deterministic synthetic inputs (restated bit for bit by oracle/oracle.py).
hipError_t launch_synth_f32(float* out, int n_rows, int64_t ld, int64_t p, uint64_t seed,
                            uint64_t stream_id, int64_t row0, int64_t idx0, float scale,
                            hipStream_t s);
hipError_t launch_synth_shares(int64_t* out, int n_clients, int n_parties, int64_t ld, int64_t p,
                               uint64_t seed, int64_t client0, int64_t idx0, float enc_scale,
                               hipStream_t s);

constexpr uint64_t STREAM_DIFF = 0, STREAM_CKPT = 1, STREAM_SECRET = 2, STREAM_SHARE = 3;
constexpr float DIFF_SCALE = 2.6429e-7f;
constexpr float CKPT_SCALE = 1.32145e-6f;

}  // namespace pgh
