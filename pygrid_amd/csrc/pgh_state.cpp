// Protobuf wire walker for the syft State message (see pgh_state.h for the schema caveat).
#include "pgh_state.h"

#include <cstring>

#include <emmintrin.h>

#include "../../include/pgh_api.h"

namespace pgh_state {
namespace {

struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;

    bool varint(uint64_t* v) {
        uint64_t x = 0;
        for (int shift = 0; shift < 64; shift += 7) {
            if (p >= end) return ok = false;
            const uint8_t b = *p++;
            x |= (uint64_t)(b & 0x7F) << shift;
            if (!(b & 0x80)) { *v = x; return true; }
        }
        return ok = false;
    }
    // Skip one field of wire type wt.
    bool skip(uint32_t wt) {
        uint64_t v;
        switch (wt) {
        case 0: return varint(&v);
        case 1: if (end - p < 8) return ok = false; p += 8; return true;
        case 2: if (!varint(&v) || (uint64_t)(end - p) < v) return ok = false; p += v; return true;
        case 5: if (end - p < 4) return ok = false; p += 4; return true;
        default: return ok = false;  // groups (3/4) are not used by proto3
        }
    }
    bool len_delim(const uint8_t** b, const uint8_t** e) {
        uint64_t v;
        if (!varint(&v) || (uint64_t)(end - p) < v) return ok = false;
        *b = p;
        *e = p + v;
        p += v;
        return true;
    }
};

// Walk a message; call f(field, wiretype, reader) for each field; f must consume the value.
template <class F>
bool each_field(const uint8_t* b, const uint8_t* e, F&& f) {
    Reader r{b, e};
    while (r.p < r.end) {
        uint64_t key;
        if (!r.varint(&key)) return false;
        const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
        if (field == 0) return false;
        if (!f(field, wt, r)) return false;
    }
    return r.ok;
}

bool parse_size(const uint8_t* b, const uint8_t* e, std::vector<int64_t>* dims) {
    return each_field(b, e, [&](uint32_t f, uint32_t wt, Reader& r) {
        if (f == SIZE_DIMS && wt == 2) {  // packed int32
            const uint8_t *pb, *pe;
            if (!r.len_delim(&pb, &pe)) return false;
            Reader q{pb, pe};
            while (q.p < q.end) {
                uint64_t v;
                if (!q.varint(&v)) return false;
                dims->push_back((int64_t)(int32_t)(uint32_t)v);
            }
            return true;
        }
        if (f == SIZE_DIMS && wt == 0) {
            uint64_t v;
            if (!r.varint(&v)) return false;
            dims->push_back((int64_t)(int32_t)(uint32_t)v);
            return true;
        }
        return r.skip(wt);
    });
}

bool parse_tensor_data(const uint8_t* base, const uint8_t* b, const uint8_t* e, Span* s, std::string* msg) {
    bool have_f32 = false, have_i64 = false;
    bool ok = each_field(b, e, [&](uint32_t f, uint32_t wt, Reader& r) {
        const uint8_t *pb, *pe;
        if (f == TD_SHAPE && wt == 2) {
            if (!r.len_delim(&pb, &pe)) return false;
            s->shape.clear();
            return parse_size(pb, pe, &s->shape);
        }
        if (f == TD_DTYPE && wt == 2) {
            if (!r.len_delim(&pb, &pe)) return false;
            s->dtype.assign((const char*)pb, (size_t)(pe - pb));
            return true;
        }
        if (f == TD_F32) {
            if (wt != 2) { *msg = "unpacked float32 payload is not supported"; return false; }
            if (have_f32) { *msg = "float32 payload split over several fields"; return false; }
            if (!r.len_delim(&pb, &pe)) return false;
            if ((pe - pb) % 4) { *msg = "float32 payload length is not a multiple of 4"; return false; }
            if (have_i64) { *msg = "tensor holds both float32 and int64 payloads"; return false; }
            s->offset = (size_t)(pb - base);
            s->count = (pe - pb) / 4;
            s->nbytes = (size_t)(pe - pb);
            have_f32 = true;
            return true;
        }
        if (f == TD_I64) {
            if (wt != 2) { *msg = "unpacked int64 payload is not supported"; return false; }
            if (have_i64) { *msg = "int64 payload split over several fields"; return false; }
            if (have_f32) { *msg = "tensor holds both float32 and int64 payloads"; return false; }
            if (!r.len_delim(&pb, &pe)) return false;
            s->offset = (size_t)(pb - base);
            s->nbytes = (size_t)(pe - pb);
            s->i64 = true;
            have_i64 = true;
            return true;
        }
        return r.skip(wt);
    });
    if (ok && have_i64) {  // element count comes from the shape; the varint pass checks the payload
        int64_t numel = 1;
        for (auto d : s->shape) numel *= d;
        s->count = s->shape.empty() ? -1 : numel;
    }
    if (ok && !have_f32 && !have_i64) {
        // proto3 omits an empty packed field: a zero-element tensor has no payload
        int64_t numel = 1;
        for (auto d : s->shape) numel *= d;
        if (s->shape.empty() || numel != 0) { *msg = "tensor has no float32 payload (dtype '" + s->dtype + "')"; return false; }
        s->offset = (size_t)(e - base);
        s->count = 0;
    }
    return ok;
}

bool parse_torch_tensor(const uint8_t* base, const uint8_t* b, const uint8_t* e, Span* s, std::string* msg) {
    bool found = false;
    bool ok = each_field(b, e, [&](uint32_t f, uint32_t wt, Reader& r) {
        if (f == TORCH_CONTENTS_DATA && wt == 2) {
            const uint8_t *pb, *pe;
            if (!r.len_delim(&pb, &pe)) return false;
            found = true;
            return parse_tensor_data(base, pb, pe, s, msg);
        }
        return r.skip(wt);
    });
    if (ok && !found) { if (msg->empty()) *msg = "TorchTensor without contents_data (binary serializer?)"; return false; }
    return ok;
}

bool parse_state_tensor(const uint8_t* base, const uint8_t* b, const uint8_t* e, Span* s, std::string* msg) {
    bool found = false;
    bool ok = each_field(b, e, [&](uint32_t f, uint32_t wt, Reader& r) {
        const uint8_t *pb, *pe;
        if (f == STATETENSOR_TORCH && wt == 2) {
            if (!r.len_delim(&pb, &pe)) return false;
            found = true;
            return parse_torch_tensor(base, pb, pe, s, msg);
        }
        if (f == STATETENSOR_PARAM && wt == 2) {
            if (!r.len_delim(&pb, &pe)) return false;
            return each_field(pb, pe, [&](uint32_t f2, uint32_t wt2, Reader& r2) {
                if (f2 == PARAM_TENSOR && wt2 == 2) {
                    const uint8_t *qb, *qe;
                    if (!r2.len_delim(&qb, &qe)) return false;
                    found = true;
                    return parse_torch_tensor(base, qb, qe, s, msg);
                }
                return r2.skip(wt2);
            });
        }
        return r.skip(wt);
    });
    if (ok && !found) { if (msg->empty()) *msg = "StateTensor holds neither torch_tensor nor torch_param"; return false; }
    return ok;
}

}  // namespace

int walk(const uint8_t* pb, size_t n, std::vector<Span>* spans, std::string* msg) {
    spans->clear();
    msg->clear();
    if (!pb && n) { *msg = "null buffer"; return PGH_E_PARSE; }
    const uint8_t* base = pb;
    bool ok = each_field(pb, pb + n, [&](uint32_t f, uint32_t wt, Reader& r) {
        if (f == STATE_TENSORS && wt == 2) {
            const uint8_t *b, *e;
            if (!r.len_delim(&b, &e)) return false;
            Span s;
            if (!parse_state_tensor(base, b, e, &s, msg)) return false;
            spans->push_back(std::move(s));
            return true;
        }
        return r.skip(wt);
    });
    if (!ok) {
        if (msg->empty()) *msg = "truncated or malformed protobuf";
        return PGH_E_PARSE;
    }
    return 0;
}

int scan(const uint8_t* pb, size_t n, std::vector<Span>* spans, std::string* msg) {
    int rc = walk(pb, n, spans, msg);
    if (rc) return rc;
    for (size_t t = 0; t < spans->size(); ++t) {
        const Span& s = (*spans)[t];
        if (s.i64) {
            *msg = "tensor " + std::to_string(t) + " holds an int64 payload, expected float32";
            return PGH_E_PARSE;
        }
        int64_t numel = 1;
        for (auto d : s.shape) {
            if (d < 0) { *msg = "negative dimension in tensor " + std::to_string(t); return PGH_E_PARSE; }
            numel *= d;
        }
        if (!s.shape.empty() && numel != s.count) {
            *msg = "tensor " + std::to_string(t) + ": shape holds " + std::to_string(numel) + " elements, payload " +
                   std::to_string(s.count);
            return PGH_E_PARSE;
        }
        if (!s.dtype.empty() && s.dtype != "float32" && s.dtype != "torch.float32") {
            *msg = "tensor " + std::to_string(t) + " has dtype '" + s.dtype + "', expected float32";
            return PGH_E_PARSE;
        }
    }
    return 0;
}

int scan_i64(const uint8_t* pb, size_t n, std::vector<Span>* spans, std::string* msg) {
    int rc = walk(pb, n, spans, msg);
    if (rc) return rc;
    for (size_t t = 0; t < spans->size(); ++t) {
        Span& s = (*spans)[t];
        for (auto d : s.shape)
            if (d < 0) { *msg = "negative dimension in tensor " + std::to_string(t); return PGH_E_PARSE; }
        if (!s.i64 && s.nbytes) {
            *msg = "tensor " + std::to_string(t) + " holds a float32 payload, expected int64 shares";
            return PGH_E_PARSE;
        }
        if (!s.dtype.empty() && s.dtype != "int64" && s.dtype != "torch.int64") {
            *msg = "tensor " + std::to_string(t) + " has dtype '" + s.dtype + "', expected int64";
            return PGH_E_PARSE;
        }
    }
    return 0;
}

namespace {
// Varint statistics of 64-byte blocks (bit j of a block mask = byte j has bit 7 set, i.e. is a
// continuation byte; SSE2 movemask, x86-64 baseline).  COPY also streams the block to dst with
// non-temporal stores (dst 16-byte aligned): one read of the source for the staging copy and the
// count together, and no read-for-ownership of the destination.
template <bool COPY>
VarintStats stats_impl(uint8_t* dst, const uint8_t* p, size_t n) {
    VarintStats st;
    int64_t run = 0;        // continuation bytes since the last terminator
    bool seen = false;      // a terminator seen yet
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i + 48));
        if (COPY) {
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
        }
        const uint64_t m = (uint64_t)(uint32_t)_mm_movemask_epi8(a) | (uint64_t)(uint32_t)_mm_movemask_epi8(b) << 16 |
                           (uint64_t)(uint32_t)_mm_movemask_epi8(c) << 32 | (uint64_t)(uint32_t)_mm_movemask_epi8(d) << 48;
        if (m == ~0ull) { run += 64; if (run > 9) st.overlong = true; continue; }
        const uint64_t t = ~m;
        const int lead = __builtin_ctzll(t);  // continuation bytes before the first terminator here
        if (run + lead > 9) st.overlong = true;
        if (!seen) { st.lead = run + lead; seen = true; }
        // runs of >= 10 continuation bytes strictly inside the 64 (the top run is carried on)
        const uint64_t r2 = m & (m >> 1), r4 = r2 & (r2 >> 2), r8 = r4 & (r4 >> 4);  // bit j: j..j+1/3/7 set
        if (r8 & (r2 >> 8)) st.overlong = true;                                        // j..j+9 set
        st.terminators += __builtin_popcountll(t);
        run = __builtin_clzll(t);
    }
    if (COPY) {
        if (i < n) std::memcpy(dst + i, p + i, n - i);
        _mm_sfence();
    }
    for (; i < n; ++i) {
        if (p[i] & 0x80) { if (++run > 9) st.overlong = true; continue; }
        if (!seen) { st.lead = run; seen = true; }
        st.terminators += 1;
        run = 0;
    }
    if (!seen) st.lead = run;
    st.trail = run;
    return st;
}
}  // namespace

VarintStats varint_stats(const uint8_t* p, size_t n) { return stats_impl<false>(nullptr, p, n); }

VarintStats varint_copy_stats(uint8_t* dst, const uint8_t* src, size_t n) {
    if (reinterpret_cast<uintptr_t>(dst) & 15) {
        std::memcpy(dst, src, n);
        return stats_impl<false>(nullptr, dst, n);
    }
    return stats_impl<true>(dst, src, n);
}

int decode_f32(const uint8_t* pb, size_t n, const std::vector<int64_t>& numel, float* out, std::string* msg) {
    std::vector<Span> spans;
    int rc = scan(pb, n, &spans, msg);
    if (rc) return rc;
    if (spans.size() != numel.size()) {
        *msg = "State holds " + std::to_string(spans.size()) + " tensors, layout has " + std::to_string(numel.size());
        return PGH_E_PARSE;
    }
    size_t off = 0;
    for (size_t t = 0; t < spans.size(); ++t) {
        if (spans[t].count != numel[t]) {
            *msg = "tensor " + std::to_string(t) + " holds " + std::to_string(spans[t].count) + " floats, layout " +
                   std::to_string(numel[t]);
            return PGH_E_PARSE;
        }
        std::memcpy(out + off, pb + spans[t].offset, 4 * (size_t)spans[t].count);  // little-endian fixed32
        off += (size_t)spans[t].count;
    }
    return 0;
}

}  // namespace pgh_state

// ---- C ABI for the codec (host only; used by the Python mirror of model_manager) ----------
extern "C" {

// Count tensors and fill up to `cap` entries of (payload byte offset, element count).
int pgh_state_scan(const uint8_t* pb, size_t n, int cap, int64_t* offsets, int64_t* counts, int* n_tensors) {
    if (!n_tensors) return PGH_E_ARG;
    std::vector<pgh_state::Span> spans;
    std::string msg;
    int rc = pgh_state::scan(pb, n, &spans, &msg);
    if (rc) return rc;
    *n_tensors = (int)spans.size();
    for (int t = 0; t < cap && t < (int)spans.size(); ++t) {
        if (offsets) offsets[t] = (int64_t)spans[t].offset;
        if (counts) counts[t] = spans[t].count;
    }
    return PGH_OK;
}

// int64 shares: per tensor the payload byte range and the number of packed varints it holds,
// validated like protobuf's parser would (no varint longer than 10 bytes, none cut off at the
// end of the payload, the count equal to the shape's element count when a shape is given).
int pgh_state_scan_i64(const uint8_t* pb, size_t n, int cap, int64_t* offsets, int64_t* nbytes, int64_t* counts,
                       int* n_tensors) {
    if (!n_tensors) return PGH_E_ARG;
    std::vector<pgh_state::Span> spans;
    std::string msg;
    int rc = pgh_state::scan_i64(pb, n, &spans, &msg);
    if (rc) return rc;
    *n_tensors = (int)spans.size();
    for (int t = 0; t < (int)spans.size(); ++t) {
        const auto& s = spans[t];
        const pgh_state::VarintStats st = pgh_state::varint_stats(pb + s.offset, s.nbytes);
        if (st.overlong || st.trail) return PGH_E_PARSE;
        if (s.count >= 0 && st.terminators != s.count) return PGH_E_PARSE;
        if (t < cap) {
            if (offsets) offsets[t] = (int64_t)s.offset;
            if (nbytes) nbytes[t] = (int64_t)s.nbytes;
            if (counts) counts[t] = st.terminators;
        }
    }
    return PGH_OK;
}

// New checkpoint bytes = `tmpl` (the current checkpoint) with every tensor payload replaced by
// `values` (concatenated, P floats).  `out` has room for n bytes (the size never changes).
int pgh_state_patch(const uint8_t* tmpl, size_t n, const float* values, int64_t n_values, uint8_t* out) {
    if (!tmpl || !out || (!values && n_values)) return PGH_E_ARG;
    std::vector<pgh_state::Span> spans;
    std::string msg;
    int rc = pgh_state::scan(tmpl, n, &spans, &msg);
    if (rc) return rc;
    int64_t total = 0;
    for (auto& s : spans) total += s.count;
    if (total != n_values) return PGH_E_ARG;
    // Spans in message order and disjoint (the walker's output for any well-formed State): copy
    // the template bytes between them (the framing) and the new payloads into them, every output
    // byte written once.  Anything else: copy the whole template first.
    bool ordered = true;
    for (size_t t = 1; t < spans.size(); ++t)
        ordered = ordered && spans[t].offset >= spans[t - 1].offset + 4 * (size_t)spans[t - 1].count;
    if (!ordered && out != tmpl) std::memcpy(out, tmpl, n);
    if (!ordered) tmpl = out;  // framing already in place
    size_t pos = 0;
    int64_t off = 0;
    for (auto& s : spans) {
        if (out != tmpl && s.offset > pos) std::memcpy(out + pos, tmpl + pos, s.offset - pos);
        std::memcpy(out + s.offset, values + off, 4 * (size_t)s.count);
        off += s.count;
        pos = s.offset + 4 * (size_t)s.count;
    }
    if (out != tmpl && n > pos) std::memcpy(out + pos, tmpl + pos, n - pos);
    return PGH_OK;
}

}  // extern "C"

// ---- fresh checkpoint framing (serialize_model_params, model_manager.py:79-92) -----------------------
namespace {
void put_varint(std::string* o, uint64_t v) {
    while (v >= 0x80) {
        o->push_back((char)(uint8_t)(v | 0x80));
        v >>= 7;
    }
    o->push_back((char)(uint8_t)v);
}
void put_key(std::string* o, uint32_t field, uint32_t wt) { put_varint(o, ((uint64_t)field << 3) | wt); }
void put_bytes(std::string* o, uint32_t field, const std::string& b) {
    put_key(o, field, 2);
    put_varint(o, b.size());
    o->append(b);
}
std::string id_msg(int64_t id) {  // Id{id_int = 2}; proto3 omits a zero id
    std::string m;
    if (id) {
        put_key(&m, 2, 0);
        put_varint(&m, (uint64_t)id);
    }
    return m;
}
size_t varint_len(uint64_t v) {
    size_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}
constexpr int SERIALIZER_ALL = 4;  // TorchTensor.serializer as state_schema.SERIALIZER_ALL
}  // namespace

extern "C" int pgh_state_fresh(const uint8_t* tmpl, size_t n, const int64_t* ids, int n_ids, uint8_t* out, size_t cap,
                               size_t* needed) {
    if (!needed || (!tmpl && n)) return PGH_E_ARG;
    std::vector<pgh_state::Span> spans;
    std::string msg;
    int rc = pgh_state::scan(tmpl, n, &spans, &msg);
    if (rc) return rc;
    const size_t T = spans.size();
    if (n_ids != (int)(2 * T) || (T && !ids)) return PGH_E_ARG;
    // State.placeholders: Placeholder{id} per tensor (PlaceHolder().instantiate(p): no tags)
    std::string head;
    for (size_t k = 0; k < T; ++k) {
        std::string ph;
        put_bytes(&ph, 1, id_msg(ids[2 * k]));
        put_bytes(&head, 1, ph);
    }
    // State.tensors: StateTensor.torch_tensor{id, serializer, contents_data{shape, dtype, f32}}; the
    // payload is the last field of every enclosing message, so each tensor is prefix + payload
    std::vector<std::string> prefix(T);
    size_t total = head.size();
    for (size_t k = 0; k < T; ++k) {
        const auto& sp = spans[k];
        std::vector<int64_t> dims = sp.shape;
        int64_t numel = 1;
        for (auto d : dims) numel *= d;
        if (dims.empty() && sp.count != 1) dims.push_back(sp.count), numel = sp.count;  // no Size: 1-D
        if (numel != sp.count) return PGH_E_PARSE;
        const uint64_t pay = 4 * (uint64_t)sp.count;
        std::string size_msg, td_head;
        std::string packed;
        for (auto d : dims) put_varint(&packed, (uint64_t)(uint32_t)(int32_t)d);
        if (!packed.empty()) put_bytes(&size_msg, 1, packed);
        put_bytes(&td_head, 1, size_msg);
        put_bytes(&td_head, 2, "float32");
        std::string td_pay;
        if (pay) {
            put_key(&td_pay, 12, 2);
            put_varint(&td_pay, pay);
        }
        const uint64_t td_len = td_head.size() + td_pay.size() + pay;
        std::string tt_head;
        put_bytes(&tt_head, 1, id_msg(ids[2 * k + 1]));
        put_key(&tt_head, 2, 0);
        put_varint(&tt_head, SERIALIZER_ALL);
        put_key(&tt_head, 4, 2);
        put_varint(&tt_head, td_len);
        const uint64_t tt_len = tt_head.size() + td_len;
        const uint64_t st_len = 1 + varint_len(tt_len) + tt_len;
        std::string& pf = prefix[k];
        put_key(&pf, 2, 2);
        put_varint(&pf, st_len);
        put_key(&pf, 1, 2);
        put_varint(&pf, tt_len);
        pf += tt_head;
        pf += td_head;
        pf += td_pay;
        total += pf.size() + pay;
    }
    *needed = total;
    if (!out) return PGH_OK;
    if (cap < total) return PGH_E_ARG;
    size_t pos = 0;
    std::memcpy(out, head.data(), head.size());
    pos = head.size();
    for (size_t k = 0; k < T; ++k) {  // the payload bytes are left for the caller (pgh_ckpt_patch_state)
        std::memcpy(out + pos, prefix[k].data(), prefix[k].size());
        pos += prefix[k].size() + 4 * (size_t)spans[k].count;
    }
    return PGH_OK;
}

