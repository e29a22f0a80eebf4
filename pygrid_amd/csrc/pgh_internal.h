// Internal interface between the single-GPU context (pgh_api.cpp, pgh_ingest.cpp, pgh_reduce.cpp,
// pgh_slots.cpp) and the multi-GPU group driver (pgh_group.cpp).
// Not installed; the public surface is include/pgh_api.h.
//
// A group context (pgh_create_group) is a pgh_ctx whose `grp` is set: every public entry point
// hands it to pgh_group::* below, which drives one child pgh_ctx per GPU through the same public
// entry points, plus the few per-context internals declared here.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/pgh_api.h"

struct pgh_group;

namespace pgh_int {
int fail(pgh_ctx* c, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
pgh_group* group_of(const pgh_ctx* c);
pgh_ctx* new_group_ctx(pgh_group* g, int device);  // a context shell that owns `g`
void free_group_ctx(pgh_ctx* c);                    // the shell only (the group is freed by its owner)

// per-context internals the group driver uses
int device_of(const pgh_ctx* c);
hipStream_t stream_of(const pgh_ctx* c);
// [P_shard] device vectors at least n elements long from the next pgh_reserve on (collectives send
// equal padded shards).
int set_vec_min(pgh_ctx* c, int64_t n);
// Host copy threads of the context's staging pool (a group splits the host between its GPUs).
int set_copy_threads(pgh_ctx* c, int n);
// Synthetic inputs of local client k are generated as global client base + k (client-sharded groups).
int set_client_base(pgh_ctx* c, int64_t base);
enum Vec { V_CKPT = 0, V_SUM = 1, V_DEC = 2 };
void* vec(pgh_ctx* c, int which);
// CPUs this process may use: its affinity mask capped by a cgroup CPU quota (cgroup v2 cpu.max or
// v1 cfs_quota/period) -- a GPU lease's share of a bigger machine, which hardware_concurrency()
// (every online CPU) does not see.  Computed once.
int usable_cpus();
// Write only this shard's slice of every payload of `tmpl` into `out` (from the resident checkpoint);
// the caller writes the framing.  Pre-faults the shard's own part of `out` while the first DMA flies.
int patch_payloads(pgh_ctx* c, const uint8_t* tmpl, size_t n, uint8_t* out);
}  // namespace pgh_int

// Group driver entry points (pgh_group.cpp), one per public call that a group context accepts.
namespace pgh_group_api {
void destroy(pgh_ctx* c);
int set_layout(pgh_ctx* c, int n_tensors, const int64_t* numel);
int set_shard(pgh_ctx* c, int64_t lo, int64_t hi);
int reserve(pgh_ctx* c, int max_clients, int dtype, int n_parties);
int reset(pgh_ctx* c);
int ingest_raw(pgh_ctx* c, int client, const void* flat, size_t nbytes, int dtype);
int ingest_state(pgh_ctx* c, int client, const uint8_t* pb, size_t n);
int ingest_state_shares(pgh_ctx* c, int client, int n_parties, const uint8_t* const* pbs, const size_t* ns);
int synth_fill(pgh_ctx* c, uint64_t seed, int n_clients);
int synth_ingest(pgh_ctx* c, uint64_t seed, int client0, int n);
int set_synth_kind(pgh_ctx* c, int kind);
int set_ingest_ranges(pgh_ctx* c, int on);
int set_weights(pgh_ctx* c, const float* w, int n);
int fedavg(pgh_ctx* c, int mode, const float* ckpt, float* out);
int ckpt_upload(pgh_ctx* c, const float* ckpt, size_t nbytes);
int ckpt_upload_state(pgh_ctx* c, const uint8_t* pb, size_t n);
int fedavg_resident(pgh_ctx* c, int mode);
int ckpt_download(pgh_ctx* c, float* out);
int ckpt_patch_state(pgh_ctx* c, const uint8_t* tmpl, size_t n, uint8_t* out);
int fold_slots(pgh_ctx* c, int mode, const int32_t* slots, int n, bool finish);
int fold_restart(pgh_ctx* c);
int secagg(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out);
int stream_begin(pgh_ctx* c, int kind, int fold_batch);
int stream_flush(pgh_ctx* c);
int stream_finish(pgh_ctx* c, const float* ckpt, float* out);
int stream_finish_resident(pgh_ctx* c);
int stream_finish_secagg(pgh_ctx* c, int base, int prec, int64_t* sum_out, float* dec_out);
int set_variant(pgh_ctx* c, int variant);
int effective_variant(pgh_ctx* c, int mode);
int stats(pgh_ctx* c, pgh_stats_t* out);
int reset_stats(pgh_ctx* c);
int sync(pgh_ctx* c);
}  // namespace pgh_group_api
