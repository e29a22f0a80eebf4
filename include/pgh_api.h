/* libpygrid_hip -- C ABI of the MI355X (gfx950) aggregation engine behind PyGrid Node's
 * model-centric cycle close.
 *
 * What it replaces (reference = /root/reference, read-only):
 *   CycleManager._average_plan_diffs, apps/node/src/app/main/model_centric/cycles/
 *   cycle_manager.py:219-323, the slice :240-303 -- checkpoint unserialize (:240), per-diff
 *   unserialize (:247-250), hosted iterative avg plan (:266-269), hard-coded mean
 *   (:276-288), apply (:293-296) -- plus the PySyft 0.2.9 Z_2^64 share sum + fixed-point
 *   decode exercised by tests/data_centric/test_basic_syft_operations.py:388-454.
 *   The reference has no FFI of its own; this ABI is what a ctypes binding in the node
 *   process binds (INTEGRATION.md shows the stub).
 *
 * Conventions: every int-returning entry point returns PGH_OK (0) or a negative pgh_status;
 * pgh_last_error() then holds the message.  Plain pointers and sizes only.  Host buffers
 * passed in are borrowed for the duration of the call.  A context is single-owner and not
 * re-entrant (the reference serialises cycle close with run_task_once,
 * apps/node/src/app/main/model_centric/tasks/cycle.py:9-25).  A context drives one GPU
 * (pgh_create) or several GPUs of one node from one process (pgh_create_group); the
 * alternative is one process (and one context) per GPU, each owning a parameter shard.
 */
#ifndef PGH_API_H
#define PGH_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGH_ABI_VERSION 10

typedef struct pgh_ctx pgh_ctx;

typedef enum {
    PGH_OK = 0,
    PGH_E_ARG = -1,        /* bad argument (null, size mismatch, out of range) */
    PGH_E_HIP = -2,        /* HIP runtime / kernel launch error */
    PGH_E_STATE = -3,      /* call order / missing clients / layout not set */
    PGH_E_OOM = -4,        /* device or pinned allocation failed */
    PGH_E_PARSE = -5,      /* malformed State protobuf bytes */
    PGH_E_UNSUPPORTED = -6
} pgh_status;

/* Averaging mode.  PGH_MEAN: hard-coded path, cycle_manager.py:276-288.
 * PGH_ITERATIVE_MEAN: hosted iterative avg_plan, cycle_manager.py:266-269 with the plan of
 * examples/model-centric/01-Create-plan.ipynb:450-454.  PGH_WEIGHTED_MEAN: north_star's
 * weighted FedAvg (no reference counterpart; equals PGH_MEAN bit for bit at w == 1). */
typedef enum { PGH_MEAN = 0, PGH_ITERATIVE_MEAN = 1, PGH_WEIGHTED_MEAN = 2 } pgh_mode;
/* Stream kind for pgh_stream_begin besides the three averaging modes. */
#define PGH_STREAM_SECAGG 16

typedef enum { PGH_F32 = 0, PGH_I64 = 1 } pgh_dtype;

typedef struct {
    double kernel_ms_last;     /* duration of the last reduction kernel (HIP events) */
    double kernel_ms_total;    /* sum over timed launches since the last reset */
    uint64_t kernel_launches;  /* timed launches since the last reset */
    uint64_t kernel_bytes_last;/* algorithmic bytes of the last reduction launch */
    uint64_t kernel_bytes_total;/* algorithmic bytes over timed launches since the last reset */
    double h2d_ms_total;       /* ingest wall time (host buffer -> HBM), ms */
    uint64_t h2d_bytes_total;  /* bytes moved host -> HBM by ingest */
    double close_ms_last;      /* wall time of the last pgh_fedavg / pgh_secagg (host in/out) */
    int64_t p_shard;           /* params in this context's shard */
    int64_t ld;                /* slab block width = row stride inside a block (elements) */
    int64_t n_folded;          /* stream mode: clients folded into the running state */
    int32_t n_clients;         /* clients ingested since the last reset */
    int32_t max_clients;       /* slab capacity (slots) */
    double kernel_busy_ms_total;/* union of the timed launches' [start, end] intervals: launches
                                 * running concurrently on several streams count once */
    uint64_t h2d_staged_bytes_total; /* of h2d_bytes_total: bytes host threads first copied into
                                 * the pinned staging ring (pageable sources); page-locked sources
                                 * (pgh_host_alloc) are DMA'd as they lie and do not count */
    uint64_t d2h_bytes_total;   /* ABI 10: bytes moved HBM -> host through the D2H ring (results) */
    uint64_t d2h_kernel_bytes_total; /* ABI 10: of d2h_bytes_total, moved by a kernel instead of an
                                 * SDMA copy -- 0 since K6 k_copy_to_host was removed (r06s: it
                                 * read FINAL ranges before they had run); kept for the layout */
} pgh_stats_t;

/* ---- context lifecycle ------------------------------------------------------------------ */
int pgh_abi_version(void);
int pgh_device_count(int* n);
/* Bind a context to GPU `device`, with a pinned host staging ring of `pinned_bytes` total
 * (0 = default 256 MiB, split into 2 slots).  Also warms the device up (one small kernel launch
 * and a host -> HBM -> host copy; PGH_WARMUP=0 skips it) so the node's first cycle close does not
 * pay for the code-object load and the copy engines' first use. */
int pgh_create(int device, size_t pinned_bytes, pgh_ctx** out);
void pgh_destroy(pgh_ctx* ctx);

/* ---- several GPUs of one node in ONE process ----------------------------
 * The node closes a cycle from one thread of one process (apps/node/src/app/__init__.py:196-199,
 * tasks/cycle.py:9-25), so the library itself drives every GPU: one context over n_gpus GPUs
 * (devices[i], or 0 .. n_gpus - 1 when devices is NULL), one child context and one host thread per
 * GPU.  The parameter axis is cut into contiguous 64-aligned shards, one per GPU; each GPU holds
 * every client for its shard, so every ingest sends each GPU its slice over its own PCIe link,
 * every fold runs on all GPUs at once, host outputs are written slice by slice, and fp32 results
 * are bit-identical to one GPU.  Secure aggregation may shard the CLIENTS instead
 * (pgh_set_client_sharding before pgh_reserve of an int64 slab): client k lives on GPU
 * k / ceil(max_clients / n_gpus), each GPU sums its clients over the whole model, the Z_2^64 sums
 * are reduce-scattered (ncclReduceScatter, uint64 SUM: exact) and each GPU decodes its slice.
 * Every entry point above and below accepts a group context, except the ones taking device
 * pointers or returning slab geometry (PGH_E_UNSUPPORTED: they name one GPU -- call them on
 * pgh_group_child).  Collectives go over RCCL (librccl.so.1, loaded at first use: ncclCommInitAll
 * over the group's devices) when the devices are distinct, else (or with PGH_RCCL=0) over peer
 * copies. */
int pgh_create_group(int n_gpus, const int* devices, size_t pinned_bytes, pgh_ctx** out);
int pgh_group_size(const pgh_ctx* ctx, int* n);              /* 1 for a single-GPU context */
int pgh_group_child(pgh_ctx* ctx, int i, pgh_ctx** child);    /* borrowed context of GPU i */
int pgh_set_client_sharding(pgh_ctx* ctx, int on);
/* All-gather the resident checkpoint into a full copy on every GPU (ncclAllGather of equal shards
 * of S = ceil(P / n_gpus) rounded up to 64 floats, or peer copies): GPU g's copy holds shard r at
 * [r * S, r * S + len_r).  d_full_out (nullable) receives one device pointer per GPU. */
int pgh_group_allgather_resident(pgh_ctx* ctx, void** d_full_out);
/* The exchange in use: 1 RCCL, 0 peer copies, -1 none yet (or not a group). */
int pgh_group_backend(pgh_ctx* ctx, int* rccl);
const char* pgh_last_error(const pgh_ctx* ctx);   /* ctx may be NULL (creation errors) */
/* Page-locked host buffers: ingest DMAs them straight to HBM (no staging copy). */
int pgh_host_alloc(size_t bytes, void** out);
int pgh_host_free(void* p);
/* Mark (on = 1) a pgh_host_alloc block of n bytes as ASYNC: an ingest of State bytes lying in it
 * returns once its DMA is queued instead of waiting for it, so the caller must pgh_host_wait(p, n)
 * before writing to or reusing the block (pgh_host_free waits by itself).  on = 0 waits, then
 * unmarks.  Unmarked page-locked memory keeps the synchronous contract. */
int pgh_host_async(void* p, size_t n, int on);
/* Wait for every DMA still reading host memory [p, p + n), queued by any context. */
int pgh_host_wait(const void* p, size_t n);
/* Fault in the pages of a (fresh, pageable) host buffer now, on up to 8 threads, so that a later
 * copy into it -- the new checkpoint's payloads at a cycle close -- takes no page faults.  Best
 * effort (Linux 5.14+ MADV_POPULATE_WRITE); always returns PGH_OK for a valid range. */
int pgh_host_prefault(void* p, size_t n);

/* ---- layout ------------------------------------------------------------------------------
 * Flat parameter vector = tensors concatenated in State order
 * (model_manager.py:94-103 state.tensors()); P = sum(numel). */
int pgh_set_layout(pgh_ctx* ctx, int n_tensors, const int64_t* numel);
/* Restrict this context to the flat range [lo, hi) (param-axis shard).  Default: [0, P). */
int pgh_set_shard(pgh_ctx* ctx, int64_t lo, int64_t hi);
/* Allocate the HBM slab: max_clients slots of the shard, dtype PGH_F32 (fp32 diffs) or
 * PGH_I64 (n_parties int64 share rows per client).  Forgets previously ingested clients.
 * RESIDENT use: client k lives in slot k (k < max_clients).  STREAM use (pgh_stream_begin):
 * client k goes to slot k % max_clients, so the slab is a ring and N may exceed it. */
int pgh_reserve(pgh_ctx* ctx, int max_clients, int dtype, int n_parties);
/* Forget ingested clients and weights (start of a new cycle); keeps allocations. */
int pgh_reset(pgh_ctx* ctx);

/* ---- ingest (the diffs of cycle_manager.py:243-250) -------------------------------------- */
/* Client `client`'s already-decoded flat diff.  PGH_F32: `flat` holds P float32 (the whole
 * model; the shard slice is taken) or P_shard float32 (this shard only).  PGH_I64: n_parties x
 * P (or x P_shard) int64 shares, party-major.  Pageable memory is staged through the pinned
 * ring; page-locked memory (pgh_host_alloc, hipHostRegister) is DMA'd directly. */
int pgh_ingest_raw(pgh_ctx* ctx, int client, const void* flat, size_t nbytes, int dtype);
/* Client diff as syft State protobuf bytes (model_manager.py:94-103 wire format, build-owned
 * schema restatement: DESIGN.md "State codec"); fp32 tensors only. */
int pgh_ingest_state(pgh_ctx* ctx, int client, const uint8_t* pb, size_t n);
/* One client's secure-aggregation shares as State bytes, one message per party (n_parties ==
 * the parties of pgh_reserve): every tensor a packed-varint contents_int64 payload, the State
 * order of pgh_set_layout (PySyft 0.2.9 int64 share tensors, test_basic_syft_operations.py:
 * 388-454; wire schema restated, parity unpinned like pgh_ingest_state).  The payload bytes go
 * to HBM as they are (PCIe carries the varints) and are decoded there (k_varint_decode); the
 * host only checks the framing, counts the values per 16 KiB chunk and rejects varints longer
 * than 10 bytes, cut-off payloads and count/layout mismatches (PGH_E_PARSE). */
int pgh_ingest_state_shares(pgh_ctx* ctx, int client, int n_parties, const uint8_t* const* pbs, const size_t* ns);
/* Fill slab rows [0, n_clients) with the deterministic synthetic diffs (or shares) of
 * SURVEY.md 8(d) for this shard, generated on the GPU (oracle/oracle.py restates them). */
int pgh_synth_fill(pgh_ctx* ctx, uint64_t seed, int n_clients);
/* Generator of the synthetic fp32 diffs for later pgh_synth_fill / pgh_synth_ingest calls:
 * 0 = one splitmix64 word per param, Irwin-Hall(4 x u16) (default); 1 = one word
 * per 4 params, a u16 each, uniform (config 4's on-device data source: write-bound instead of
 * integer-bound).  Both restated bit for bit by oracle/oracle.py. */
int pgh_set_synth_kind(pgh_ctx* ctx, int kind);
/* Ingest synthetic clients [client0, client0 + n) generated on the GPU (either use). */
int pgh_synth_ingest(pgh_ctx* ctx, uint64_t seed, int client0, int n);
/* Per-client weights for PGH_WEIGHTED_MEAN (n == clients ingested at reduction time). */
int pgh_set_weights(pgh_ctx* ctx, const float* w, int n);

/* ---- reduction ----------------------------------------------------------------------------
 * out = ckpt - avg(diffs), over this context's shard.  Host pointers, P_shard floats each. */
int pgh_fedavg(pgh_ctx* ctx, int mode, const float* ckpt, float* out);
/* Same with device pointers (16-byte aligned, P_shard floats) on caller stream `stream`
 * (a hipStream_t; NULL = the HIP default stream, ordered with other blocking streams).  Nothing
 * is copied to the host. */
int pgh_fedavg_device(pgh_ctx* ctx, int mode, const float* d_ckpt, float* d_out, void* stream);
/* Only the shard-relative param range [off, off + len) (off a multiple of 4): lets a caller
 * overlap the collective that ships finished ranges with the fold of the next one.  d_ckpt and
 * d_out are the shard base pointers. */
int pgh_fedavg_device_range(pgh_ctx* ctx, int mode, int64_t off, int64_t len, const float* d_ckpt, float* d_out,
                            void* stream);
/* ---- resident checkpoint: keep the model in HBM across cycles ---------
 * Upload the current checkpoint once (flat floats: the whole model or this shard; or straight
 * from its State bytes), fold with pgh_fedavg_resident -- the result replaces the resident
 * checkpoint, so the next cycle needs no checkpoint upload -- and read it back as floats or as
 * State bytes (the template's payload spans overwritten, like pgh_state_patch). */
int pgh_ckpt_upload(pgh_ctx* ctx, const float* ckpt, size_t nbytes);
int pgh_ckpt_upload_state(pgh_ctx* ctx, const uint8_t* pb, size_t n);
int pgh_fedavg_resident(pgh_ctx* ctx, int mode);
int pgh_ckpt_download(pgh_ctx* ctx, float* out);  /* P_shard floats */
/* out (n bytes) = tmpl with this shard's slice of every payload taken from the resident checkpoint. */
int pgh_ckpt_patch_state(pgh_ctx* ctx, const uint8_t* tmpl, size_t n, uint8_t* out);

/* ---- report-time folds of scattered slots -----------------------------
 * RESIDENT slab.  Diffs are ingested into whichever slot is free when they are reported (client
 * index = slot); the fold order is the reference's close-time order -- completed WorkerCycles in
 * assignment (row id) order, cycle_manager.py:243-245 -- which the caller gives as slot lists:
 * pgh_fold_slots folds `slots` (n entries, in list order) into the running fold state as soon as
 * their positions are certain, and frees them for new ingests; the k-th slot folded since
 * pgh_reset / pgh_reserve is fold client k (the iterative plan's k, weight index k; weights are set
 * in fold order with pgh_set_weights).  pgh_fold_slots_finish_resident folds the rest (n may be 0)
 * and writes ckpt - avg into the resident checkpoint (pgh_ckpt_upload*), like
 * pgh_fedavg_resident: bit-identical to folding every diff contiguously at close.  `mode` stays the
 * same within a cycle. */
int pgh_fold_slots(pgh_ctx* ctx, int mode, const int32_t* slots, int n);
int pgh_fold_slots_finish_resident(pgh_ctx* ctx, int mode, const int32_t* slots, int n);
/* Discard the running fold state of this cycle's slot folds (the diffs folded so far are gone
 * from it; the next pgh_fold_slots starts again at fold client 0, and weights must be set again).
 * Slots holding unfolded diffs keep them.  Used when the close-time order of the
 * completed WorkerCycles (cycle_manager.py:243-245) differs from the order the early folds
 * assumed, or a folded worker re-reported (submit_worker_diff overwrites its diff, :162-174):
 * the caller then re-folds every diff in the query's order, bit-identical to the reference. */
int pgh_fold_slots_restart(pgh_ctx* ctx);
/* Report-time ingest (on != 0; default off): every State diff of a shard of >= 1M params is
 * copied to HBM in param ranges with an event each, and the close's fold
 * (pgh_fold_slots_finish_resident) starts each range as soon as the LAST report's copy of that
 * range has landed instead of waiting for the whole copy -- the close overlaps the tail of the
 * last report's DMA.  Costs a few % of H2D throughput per diff (more, smaller copies), so it is
 * for report-time aggregation, not for a close that ingests every diff at once. */
int pgh_set_ingest_ranges(pgh_ctx* ctx, int on);

/* Z_2^64 share sum over all clients x parties, then decode float32(sum) / base**prec.
 * sum_out (int64) and dec_out (float32) are host arrays of P_shard; either may be NULL. */
int pgh_secagg(pgh_ctx* ctx, int base, int prec, int64_t* sum_out, float* dec_out);
int pgh_secagg_device(pgh_ctx* ctx, int base, int prec, int64_t* d_sum, float* d_dec, void* stream);
/* Only the shard-relative param range [off, off + len) (off % 4 == 0); d_sum / d_dec are the
 * shard-sized outputs, of which only that range is written (multi-GPU gather overlap). */
int pgh_secagg_device_range(pgh_ctx* ctx, int base, int prec, int64_t off, int64_t len, int64_t* d_sum,
                            float* d_dec, void* stream);
/* Decode only: d_dec[i] = float32(int64 d_sum[i]) / base**prec for i < n, on `stream` (device
 * pointers; needs no slab).  Client-sharded secure aggregation: every rank sums the shares of its
 * own clients (pgh_secagg_device with d_dec = NULL), the [P] sums are reduce-scattered with an
 * int64 SUM (wrap-add is associative: exact), and each rank decodes its param shard here -- the
 * same expression as pgh_secagg's decode.  Replaces the decode half of PySyft 0.2.9's
 * FixedPrecisionTensor.float_precision (test_basic_syft_operations.py:417-424). */
int pgh_secagg_decode_device(pgh_ctx* ctx, int base, int prec, const int64_t* d_sum, int64_t n, float* d_dec,
                             void* stream);
/* Fill a device buffer with the synthetic checkpoint of this shard (P_shard floats). */
int pgh_synth_ckpt_device(pgh_ctx* ctx, uint64_t seed, float* d_ckpt, void* stream);

/* ---- STREAM use: fold clients in order as they arrive ---------------------------------------
 * After pgh_stream_begin, every run of >= fold_batch consecutive clients at the fold front is
 * folded into the running state (same op order as RESIDENT: bit-identical results) and its slots
 * are freed; H2D of later clients overlaps those folds.  kind = a pgh_mode or PGH_STREAM_SECAGG;
 * fold_batch <= 0 means half the slots.  Clients may arrive out of order within the ring. */
int pgh_stream_begin(pgh_ctx* ctx, int kind, int fold_batch);
int pgh_stream_flush(pgh_ctx* ctx);               /* fold the ready run now */
/* Fold what is left and write out = ckpt - avg (all clients [0, n) must have arrived). */
int pgh_stream_finish(pgh_ctx* ctx, const float* ckpt, float* out);
int pgh_stream_finish_device(pgh_ctx* ctx, const float* d_ckpt, float* d_out, void* stream);
/* Finish into the resident checkpoint (pgh_ckpt_upload / pgh_ckpt_upload_state, possibly uploaded
 * while clients were still arriving): afterwards it IS the new checkpoint, ready for
 * pgh_ckpt_patch_state / pgh_ckpt_download and the next cycle. */
int pgh_stream_finish_resident(pgh_ctx* ctx);
int pgh_stream_finish_secagg(pgh_ctx* ctx, int base, int prec, int64_t* sum_out, float* dec_out);
int pgh_stream_finish_secagg_device(pgh_ctx* ctx, int base, int prec, int64_t* d_sum, float* d_dec, void* stream);

/* ---- tuning and observability -------------------------------------------------------------- */
/* Kernel variant for A/B measurement (table in csrc/pgh_kernels.hip); -1 = the default, which
 * picks by shard size (auto_variant in csrc/pgh_kernels.hip). */
#define PGH_DEFAULT_VARIANT (-1)
int pgh_set_variant(pgh_ctx* ctx, int variant);
/* The variant the next fold of this context's shard runs for `mode` (a pgh_mode, or
 * PGH_STREAM_SECAGG for the share sum): >= 0, or an error status. */
int pgh_effective_variant(pgh_ctx* ctx, int mode);
int pgh_stats(pgh_ctx* ctx, pgh_stats_t* out);     /* synchronises pending timing events */
int pgh_reset_stats(pgh_ctx* ctx);
/* Device pointer and geometry of the slab, for callers that drive the kernels.  The slab is
 * column-blocked: element (row r, shard param i) is at
 *   d_slab[(i / ld) * block_pitch + r * ld + i % ld]
 * (row r = slot * n_parties + party).  A shard of at most one block has block_pitch 0 and is
 * plain row-major [rows][ld]. */
int pgh_slab(pgh_ctx* ctx, void** d_slab, int64_t* ld, int64_t* block_pitch);
int pgh_sync(pgh_ctx* ctx);                       /* wait for the context's streams */

/* ---- State codec (host only; replaces syft serde at model_manager.py:79-103) ------------- */
/* Locate each tensor's packed float32 payload in a State message: byte offset and element
 * count, State order.  Up to `cap` entries are written; *n_tensors = tensors found. */
int pgh_state_scan(const uint8_t* pb, size_t n, int cap, int64_t* offsets, int64_t* counts, int* n_tensors);
/* New checkpoint (serialize_model_params, model_manager.py:79-92, as used at
 * cycle_manager.py:303): `tmpl` with every payload overwritten by `values` (P floats).  `out`
 * has n bytes; out == tmpl patches in place. */
int pgh_state_patch(const uint8_t* tmpl, size_t n, const float* values, int64_t n_values, uint8_t* out);

/* Framing of the new checkpoint as serialize_model_params emits it (model_manager.py:79-92:
 * State(state_placeholders=[PlaceHolder().instantiate(p) for p in params]) of plain tensors): per
 * tensor of `tmpl` (State order, its shapes) a Placeholder{id = ids[2k]} and a
 * StateTensor.torch_tensor{id = ids[2k + 1], serializer, contents_data{shape, "float32", payload}};
 * no tags.  *needed = message bytes; with out (cap >= *needed) the framing is written and every
 * payload span left for pgh_ckpt_patch_state(ctx, out, n, out) (in place) or the caller.  n_ids must
 * be 2 x the tensors of tmpl. */
int pgh_state_fresh(const uint8_t* tmpl, size_t n, const int64_t* ids, int n_ids, uint8_t* out, size_t cap,
                    size_t* needed);

/* Secure-aggregation shares as State bytes: every tensor a TensorData.contents_int64 (packed
 * varint; build-owned schema restatement, field 10).  Per tensor: payload byte offset, payload
 * bytes and the number of int64 values, validated as protobuf's parser would (varints of at most
 * 10 bytes, none cut off, count == shape numel when a shape is present).  PGH_E_PARSE otherwise. */
int pgh_state_scan_i64(const uint8_t* pb, size_t n, int cap, int64_t* offsets, int64_t* nbytes, int64_t* counts,
                       int* n_tensors);

/* ---- report path (host only): base64 of the diff (fl_events.py:257) ----------------------- */
size_t pgh_b64_decoded_cap(size_t n);
/* Python base64.b64decode semantics (non-validating); threads <= 0 = auto.  PGH_E_PARSE on bad
 * padding. */
int pgh_b64_decode(const char* in, size_t n, uint8_t* out, size_t* written, int threads);
/* Decoded size, computed from the text after the last whole quad of the '='-free prefix alone,
 * valid IF that prefix is all alphabet characters (the common case; not checked).  PGH_E_PARSE when
 * that tail is not clean: use pgh_b64_decode(out = NULL) for the exact size then. */
int pgh_b64_clean_size(const char* in, size_t n, size_t* size);
/* One pass for a clean string (every character before the first '=' in the alphabet): `out` holds
 * `cap` = pgh_b64_clean_size bytes.  PGH_E_STATE when the text is not clean (or decodes to more than
 * cap): take pgh_b64_decode then. */
int pgh_b64_decode_clean(const char* in, size_t n, uint8_t* out, size_t cap, size_t* written, int threads);

#ifdef __cplusplus
}
#endif
#endif /* PGH_API_H */
