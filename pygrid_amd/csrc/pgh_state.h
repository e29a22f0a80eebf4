// syft State protobuf codec (host side of ingest and checkpoint emit).
//
// The reference (de)serializes diffs and checkpoints with syft 0.2.9 + syft-proto 0.5.2
// (model_manager.py:79-103): State{placeholders=1, tensors=2} -> StateTensor{torch_tensor=1 |
// torch_param=2} -> TorchTensor{contents_data=4} -> TensorData{shape=1, dtype=2,
// contents_float32=F32_FIELD}.  syft-proto is not in the image, so the field numbers below are
// a BUILD-OWNED RESTATEMENT (DESIGN.md "State codec": parity unpinned until checked against
// real client bytes).  They live only here and in pygrid_amd/state_schema.py.
//
// Rather than rebuilding messages, the codec locates the byte span of every tensor's packed
// float32 payload.  Decode = memcpy out of those spans; encode of the new checkpoint = copy the
// old checkpoint bytes and overwrite the spans (same length: fixed32 payloads), which keeps every
// id / tag / description byte-identical to what the client stack emitted.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace pgh_state {

// --- restated schema (syft-proto 0.5.2, unpinned) ---
constexpr uint32_t STATE_TENSORS = 2;         // State.tensors (repeated StateTensor)
constexpr uint32_t STATETENSOR_TORCH = 1;     // StateTensor.torch_tensor (TorchTensor)
constexpr uint32_t STATETENSOR_PARAM = 2;     // StateTensor.torch_param (Parameter)
constexpr uint32_t PARAM_TENSOR = 2;          // Parameter.tensor (TorchTensor)
constexpr uint32_t TORCH_CONTENTS_DATA = 4;   // TorchTensor.contents_data (TensorData)
constexpr uint32_t TD_SHAPE = 1;              // TensorData.shape (Size)
constexpr uint32_t TD_DTYPE = 2;              // TensorData.dtype (string)
constexpr uint32_t TD_I64 = 10;               // TensorData.contents_int64 (packed varint): secagg shares
constexpr uint32_t TD_F32 = 12;               // TensorData.contents_float32 (packed float)
constexpr uint32_t SIZE_DIMS = 1;             // Size.dims (packed int32)

struct Span {
    size_t offset = 0;          // byte offset of the first payload byte in the message
    int64_t count = 0;          // floats in the span (int64 spans: elements per Size.dims, -1 if no dims)
    bool i64 = false;           // contents_int64 (packed varint) instead of contents_float32
    size_t nbytes = 0;          // payload bytes
    std::vector<int64_t> shape; // Size.dims
    std::string dtype;          // TensorData.dtype
};

// Scan a State message; one Span per tensor, in State order.  Returns 0 or PGH_E_PARSE (-5)
// with a message.  Unpacked (one-tag-per-float) payloads are rejected: spans must be contiguous.
int scan(const uint8_t* pb, size_t n, std::vector<Span>* spans, std::string* msg);

// Scan a State whose tensors hold int64 payloads (secagg shares: TensorData.contents_int64,
// packed varint).  Same walk as scan(); spans carry the payload byte ranges.
int scan_i64(const uint8_t* pb, size_t n, std::vector<Span>* spans, std::string* msg);

// Packed-varint statistics of bytes [p, p + n) (a chunk of one payload): the number of values
// that END in it (bytes with bit 7 clear), the continuation bytes before its first terminator
// (lead) and after its last (trail; n when it has none), and whether a run of more than 9
// continuation bytes (a varint longer than 10 bytes: protobuf rejects it) lies inside.
struct VarintStats {
    int64_t terminators = 0;
    int64_t lead = 0, trail = 0;
    bool overlong = false;
};
VarintStats varint_stats(const uint8_t* p, size_t n);
// The same statistics while copying [src, src + n) to dst (non-temporal stores when dst is
// 16-byte aligned): the staging copy into the pinned ring reads each byte once.
VarintStats varint_copy_stats(uint8_t* dst, const uint8_t* src, size_t n);

// Decode every tensor into `out` (concatenated), checking per-tensor numel against `numel`.
int decode_f32(const uint8_t* pb, size_t n, const std::vector<int64_t>& numel, float* out, std::string* msg);

}  // namespace pgh_state
