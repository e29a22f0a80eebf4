// Internal launcher interface between the C-ABI context code (pgh_api.cpp, pgh_ingest.cpp,
// pgh_reduce.cpp, pgh_slots.cpp) and the gfx950 kernels (pgh_kernels.hip).
// Not installed; the public surface is include/pgh_api.h.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pgh {

// fedavg modes (same numbering as PGH_MEAN / PGH_ITERATIVE_MEAN / PGH_WEIGHTED_MEAN)
enum { MODE_MEAN = 0, MODE_ITERATIVE = 1, MODE_WEIGHTED = 2 };
// flags for a chunked (client-streaming) reduction
enum { FL_FIRST = 1, FL_FINAL = 2 };

// Column-blocked slab: the shard's params are cut into blocks of `ld`
// columns; block j holds every row's columns [j*ld, (j+1)*ld) row after row, so element
// (row r, shard param i) lives at  (i >> bshift) * bstride + r * ld + (i & bmask).
// A lane walking down the rows of one column then streams through one compact block (rows ld
// apart) instead of rows a whole shard apart.  One block (bshift = 62) is the plain row-major
// [rows][ld] layout, used for shards of at most one block and for the [p] vectors.
struct SlabMap {
    int64_t ld;        // columns per block = row stride inside a block (multiple of 4; slab: of 64)
    int64_t bstride;   // elements from block j to block j + 1 (= rows in the slab x ld)
    int bshift;        // log2(ld) when blocked, 62 for a single block
    int64_t bmask;     // ld - 1 when blocked, 2^62 - 1 for a single block
    int64_t off;       // shard param of the launch's local column 0 (range folds)
    __host__ __device__ int64_t at(int64_t local) const {
        const int64_t i = off + local;
        return (i >> bshift) * bstride + (i & bmask);
    }
};

inline SlabMap single_block(int64_t ld) { return SlabMap{ld, 0, 62, (int64_t(1) << 62) - 1, 0}; }

struct FedavgArgs {
    const float* diffs;     // slab at the first row: clients client0 .. client0+n_rows-1
    SlabMap map;            // slab geometry; map.off = shard param of local column 0
    int n_rows;
    int64_t client0;        // global index of row 0 (iterative k, weight index)
    int64_t p;              // params in this shard
    const float* weights;   // [n_rows] device, MODE_WEIGHTED only
    const double* recips;   // [n_rows] device, MODE_ITERATIVE: 1 / (double)(float)(client0 + r + 1)
    float* acc;             // [p] running state; written unless FL_FINAL
    const float* acc_in;    // [p] running state read unless FL_FIRST (nullptr: acc; a saved fold
                            // state, pgh_fold_rewind, is read from where it was saved)
    const float* ckpt;      // [p], FL_FINAL only
    float* out;             // [p], FL_FINAL only
    float divisor;          // float(N) or sum of weights, FL_FINAL of MEAN / WEIGHTED
    int flags;
    int mode;
    int variant;            // kernel variant (table in pgh_kernels.hip); < 0 = auto by shard size
};
hipError_t launch_fedavg(const FedavgArgs& a, hipStream_t s);

// Slab rows of one fold launch given by index instead of contiguous from `diffs`: row r of the
// launch is slab row rows[r] (a.diffs = the slab at row 0).  Report-time aggregation folds the
// reported diffs where they landed, in assignment order, skipping workers that never reported
// (cycle_manager.py:243-245).  Passed by value as a kernel argument (scalar loads from the
// kernarg segment), so a launch folds at most ROWTAB_MAX rows.
constexpr int ROWTAB_MAX = 512;
struct RowTab {
    int32_t rows[ROWTAB_MAX];
};
hipError_t launch_fedavg_rows(const FedavgArgs& a, const RowTab& t, hipStream_t s);

struct SecaggArgs {
    const int64_t* shares;  // slab at the first row (rows = clients x parties)
    SlabMap map;
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

// Deterministic synthetic inputs (restated bit for bit by oracle/oracle.py).  `out` is the
// slab (or a [p] vector: single_block) at its first row; params [p, ncols) are zero-filled.
hipError_t launch_synth_f32(float* out, const SlabMap& m, int64_t ncols, int n_rows, int64_t p, uint64_t seed,
                            uint64_t stream_id, int64_t row0, int64_t idx0, float scale, hipStream_t s,
                            int64_t max_wgs = 0,  // > 0: cap the grid at max_wgs workgroups
                            int kind = 0,         // 0 Irwin-Hall per param, 1 fast (4 params per word)
                            bool nt = false);     // non-temporal stores
// dec[i] = float32(int64 sum[i]) / divisor for i < n (decode after a cross-rank share-sum reduction).
hipError_t launch_secagg_decode(const int64_t* sum, float* dec, int64_t n, float divisor, hipStream_t s);
hipError_t launch_synth_shares(int64_t* out, const SlabMap& m, int64_t ncols, int n_clients, int n_parties,
                               int64_t p, uint64_t seed, int64_t client0, int64_t idx0, float enc_scale,
                               hipStream_t s);

// Packed-varint int64 payloads (secagg shares as State bytes) decoded on the GPU.  The payload
// bytes sit in HBM as received, each tensor's payload starting 16-byte aligned; they are cut into
// chunks of at most VARINT_CHUNK bytes.  `first` = index (in the flat layout) of the first value
// whose LAST byte lies in the chunk: the host counts terminator bytes per chunk while staging.
constexpr int VARINT_CHUNK = 16384;  // one wave of K4 per chunk
struct VChunk {
    int64_t off;       // chunk start, bytes from the payload buffer base (16-aligned)
    int64_t span_off;  // start of the tensor payload holding the chunk (nothing before it is read)
    int64_t first;     // flat index of the first value ending in the chunk
    int32_t n;         // bytes in the chunk
    int32_t pad;
};
// Decode every chunk into one slab row: value with flat index i goes to row[m.at(i - lo)] when
// lo <= i < hi.  Requires validated input (no varint longer than 10 bytes).
hipError_t launch_varint_decode(const uint8_t* bytes, const VChunk* chunks, int n_chunks, int64_t* row,
                                const SlabMap& m, int64_t lo, int64_t hi, hipStream_t s);

// Float payloads of a page-locked State message, DMA'd into HBM as they lie in the message (no host
// staging copy), gathered into one slab row: chunk k moves n floats starting at byte `src` of the
// buffer (any alignment: protobuf puts a payload right after its varint length) to shard elements
// dst .. dst + n - 1 of the row (row[m.at(i)]).  The buffer holds 8 readable bytes past the last
// payload byte.
constexpr int GATHER_CHUNK = 4096;
struct GChunk {
    int64_t src;
    int64_t dst;
    int32_t n;
    int32_t pad;
};
hipError_t launch_gather_f32(const uint8_t* bytes, const GChunk* chunks, int n_chunks, float* row, const SlabMap& m,
                             hipStream_t s);

constexpr uint64_t STREAM_DIFF = 0, STREAM_CKPT = 1, STREAM_SECRET = 2, STREAM_SHARE = 3;
constexpr float DIFF_SCALE = 2.6429e-7f;
constexpr float CKPT_SCALE = 1.32145e-6f;

}  // namespace pgh
