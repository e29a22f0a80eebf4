// Standard-alphabet base64 decode for the report path (host only).
//
// Reference: fl_events.report decodes every client diff with
// `base64.b64decode(data.get(CYCLE.DIFF, None).encode())` (apps/node/src/app/main/events/
// model_centric/fl_events.py:257) -- O(diff bytes) per request, 47 MB per ResNet-18 diff.
//
// Semantics are CPython 3.10's non-validating binascii.a2b_base64 (what b64decode calls with
// validate=False), which is a state machine over the characters: alphabet characters fill a
// 4-character quad; any other character except '=' is skipped; '=' is skipped unless at least two
// characters of the current quad are present, and there it counts as padding -- once quad
// position + padding reaches 4 the decode stops, ignoring the rest.  A data character resets the
// padding count.  Input that ends inside a quad is an error (1 character over: "cannot be 1 more
// than a multiple of 4", 2-3: "Incorrect padding").
//
// Fast path (the common case: one clean base64 string): every character before the first '=' is
// in the alphabet, so quad g is characters [4g, 4g + 4) and every thread decodes its own quads at
// fixed positions with AVX2 (32 characters -> 24 bytes per step: pshufb range check + translate,
// maddubs / madd bit packing; Mula's layout), falling back to the general form below at the first
// non-alphabet character anywhere.  Only the last 0-3 prefix characters and the input from the
// first '=' go through the machine.
//
// Parallel form: before the first '=' the machine only decodes alphabet characters and skips the
// rest.  A parallel count of the prefix's alphabet characters per chunk gives every chunk its
// position in that character stream; each thread then decodes the whole quads whose first
// character lies in its chunk: their characters are compacted (stray characters dropped; AVX2 +
// BMI2 pext) into a small thread-local buffer piece by piece and decoded as clean text.  The
// machine itself runs only over the prefix's last 0-3 alphabet characters and the input from the
// first '=' on.
#include <immintrin.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>

#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pgh_api.h"

namespace {

struct Table {
    int8_t v[256];
    Table() {
        std::memset(v, -1, sizeof v);
        const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
        for (int i = 0; i < 64; ++i) v[(unsigned char)a[i]] = (int8_t)i;
    }
};
const Table kT;

// Decode `n4` complete quads of alphabet characters into out; returns bytes written.
size_t decode_groups(const unsigned char* in, size_t n4, uint8_t* out) {
    for (size_t g = 0; g < n4; ++g) {
        const uint32_t x = ((uint32_t)kT.v[in[0]] << 18) | ((uint32_t)kT.v[in[1]] << 12) |
                           ((uint32_t)kT.v[in[2]] << 6) | (uint32_t)kT.v[in[3]];
        out[0] = (uint8_t)(x >> 16);
        out[1] = (uint8_t)(x >> 8);
        out[2] = (uint8_t)x;
        in += 4;
        out += 3;
    }
    return n4 * 3;
}

// CPython's a2b_base64 loop (non-strict), resumable: feed() runs characters through it and
// appends output bytes; `done` once a complete padding sequence has been seen.
struct Machine {
    int quad_pos = 0, pads = 0;
    unsigned leftchar = 0;
    bool done = false;
    void feed(const unsigned char* p, size_t n, std::vector<uint8_t>* out) {
        for (size_t i = 0; i < n && !done; ++i) {
            const unsigned char ch = p[i];
            if (ch == '=') {
                if (quad_pos >= 2 && quad_pos + ++pads >= 4) done = true;
                continue;
            }
            const int v = kT.v[ch];
            if (v < 0) continue;
            pads = 0;
            switch (quad_pos) {
            case 0: quad_pos = 1; leftchar = (unsigned)v; break;
            case 1: quad_pos = 2; out->push_back((uint8_t)((leftchar << 2) | ((unsigned)v >> 4))); leftchar = (unsigned)v & 0x0f; break;
            case 2: quad_pos = 3; out->push_back((uint8_t)((leftchar << 4) | ((unsigned)v >> 2))); leftchar = (unsigned)v & 0x03; break;
            default: quad_pos = 0; out->push_back((uint8_t)((leftchar << 6) | (unsigned)v)); leftchar = 0; break;
            }
        }
    }
};

// Decode n4 quads of characters that must all be in the alphabet; false at the first one that is
// not (the output is then incomplete).
bool decode_clean_scalar(const unsigned char* in, size_t n4, uint8_t* out) {
    for (size_t g = 0; g < n4; ++g, in += 4, out += 3) {
        const int a = kT.v[in[0]], b = kT.v[in[1]], c = kT.v[in[2]], d = kT.v[in[3]];
        if ((a | b | c | d) < 0) return false;
        const uint32_t x = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | (uint32_t)d;
        out[0] = (uint8_t)(x >> 16);
        out[1] = (uint8_t)(x >> 8);
        out[2] = (uint8_t)x;
    }
    return true;
}

// Per character c (lo = c & 15, hi = c >> 4): LUT_LO[lo] & LUT_HI[hi] != 0 exactly when c is not
// in the standard alphabet (hi 2: only '+' 0x2B and '/' 0x2F; hi 3: '0'-'9'; hi 4 / 6: not '@' / '`';
// hi 5 / 7: up to 'Z' / 'z'; every other hi nibble: bit 0x10, set in every LUT_LO entry).  Value =
// c + ROLL[hi - (c == '/')].
#define PGH_B64_LUTS                                                                                   \
    const __m256i lut_lo = _mm256_setr_epi8(0x15, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, \
                                            0x13, 0x1A, 0x1B, 0x1B, 0x1B, 0x1A, 0x15, 0x11, 0x11, 0x11, \
                                            0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x13, 0x1A, 0x1B, 0x1B, \
                                            0x1B, 0x1A);                                                  \
    const __m256i lut_hi = _mm256_setr_epi8(0x10, 0x10, 0x01, 0x02, 0x04, 0x08, 0x04, 0x08, 0x10, 0x10, \
                                            0x10, 0x10, 0x10, 0x10, 0x10, 0x10, 0x10, 0x10, 0x01, 0x02, \
                                            0x04, 0x08, 0x04, 0x08, 0x10, 0x10, 0x10, 0x10, 0x10, 0x10, \
                                            0x10, 0x10);                                                  \
    const __m256i nib = _mm256_set1_epi8(0x0f)

__attribute__((target("avx2"))) bool all_alphabet_avx2(const unsigned char* in, size_t n) {
    PGH_B64_LUTS;
    size_t i = 0;
    __m256i bad = _mm256_setzero_si256();
    for (; i + 32 <= n; i += 32) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + i));
        const __m256i hi = _mm256_and_si256(_mm256_srli_epi32(v, 4), nib);
        bad = _mm256_or_si256(bad, _mm256_and_si256(_mm256_shuffle_epi8(lut_lo, _mm256_and_si256(v, nib)),
                                                    _mm256_shuffle_epi8(lut_hi, hi)));
        if ((i & 2047) == 2016 && !_mm256_testz_si256(bad, bad)) return false;  // every 2 KiB: stop early
    }
    if (!_mm256_testz_si256(bad, bad)) return false;
    for (; i < n; ++i)
        if (kT.v[in[i]] < 0) return false;
    return true;
}

__attribute__((target("avx2"))) bool decode_clean_avx2(const unsigned char* in, size_t n4, uint8_t* out) {
    PGH_B64_LUTS;
    const __m256i lut_roll = _mm256_setr_epi8(0, 16, 19, 4, -65, -65, -71, -71, 0, 0, 0, 0, 0, 0, 0, 0, 0, 16, 19, 4,
                                              -65, -65, -71, -71, 0, 0, 0, 0, 0, 0, 0, 0);
    const __m256i slash = _mm256_set1_epi8(0x2f);
    const __m256i pack_shuf = _mm256_setr_epi8(2, 1, 0, 6, 5, 4, 10, 9, 8, 14, 13, 12, -1, -1, -1, -1, 2, 1, 0, 6, 5,
                                               4, 10, 9, 8, 14, 13, 12, -1, -1, -1, -1);
    const __m256i pack_perm = _mm256_setr_epi32(0, 1, 2, 4, 5, 6, 7, 7);
    const size_t nch = 4 * n4;
    size_t i = 0;
    for (; i + 32 <= nch; i += 32) {
        __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + i));
        const __m256i hi = _mm256_and_si256(_mm256_srli_epi32(v, 4), nib);
        const __m256i lo_b = _mm256_shuffle_epi8(lut_lo, _mm256_and_si256(v, nib));
        if (!_mm256_testz_si256(lo_b, _mm256_shuffle_epi8(lut_hi, hi))) return false;
        const __m256i roll = _mm256_shuffle_epi8(lut_roll, _mm256_add_epi8(_mm256_cmpeq_epi8(v, slash), hi));
        v = _mm256_add_epi8(v, roll);                                   // 6-bit values
        v = _mm256_maddubs_epi16(v, _mm256_set1_epi32(0x01400140));     // ab, cd (12 bits each)
        v = _mm256_madd_epi16(v, _mm256_set1_epi32(0x00011000));        // abcd (24 bits per dword)
        v = _mm256_shuffle_epi8(v, pack_shuf);                          // big-endian 3 bytes per dword
        v = _mm256_permutevar8x32_epi32(v, pack_perm);                  // 24 contiguous bytes
        uint8_t* o = out + i / 4 * 3;                                   // exactly 24 bytes: a thread
        _mm_storeu_si128(reinterpret_cast<__m128i*>(o), _mm256_castsi256_si128(v));  // never writes
        _mm_storel_epi64(reinterpret_cast<__m128i*>(o + 16), _mm256_extracti128_si256(v, 1));  // past its quads
    }
    return decode_clean_scalar(in + i, (nch - i) / 4, out + i / 4 * 3);
}

bool have_avx2() {
    static const bool yes = __builtin_cpu_supports("avx2");
    return yes;
}

// The general route's inner loops (text with characters outside the alphabet, e.g. MIME line
// breaks): AVX2 + BMI2 where the CPU has them, the scalar loops below otherwise.
bool have_avx2_bmi2() {
    static const bool yes = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi2");
    return yes;
}

// Bit j set when character j of the 32 at p is NOT in the alphabet.
__attribute__((target("avx2"))) inline uint32_t bad_mask32(const unsigned char* p) {
    PGH_B64_LUTS;
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
    const __m256i hi = _mm256_and_si256(_mm256_srli_epi32(v, 4), nib);
    const __m256i bad = _mm256_and_si256(_mm256_shuffle_epi8(lut_lo, _mm256_and_si256(v, nib)),
                                         _mm256_shuffle_epi8(lut_hi, hi));
    return ~(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(bad, _mm256_setzero_si256()));
}

// Alphabet characters in s[a, b).
__attribute__((target("avx2,popcnt"))) size_t count_alphabet_avx2(const unsigned char* s, size_t a, size_t b) {
    size_t g = 0, i = a;
    for (; i + 32 <= b; i += 32) g += 32 - (size_t)__builtin_popcount(bad_mask32(s + i));
    for (; i < b; ++i) g += kT.v[s[i]] >= 0;
    return g;
}

size_t count_alphabet(const unsigned char* s, size_t a, size_t b) {
    if (have_avx2_bmi2()) return count_alphabet_avx2(s, a, b);
    size_t g = 0;
    for (size_t i = a; i < b; ++i) g += kT.v[s[i]] >= 0;
    return g;
}

// Copy the alphabet characters of s[i, end) to dst, in order, until `want` are copied or `end` is
// reached; advances i, returns the count.  A 32-character block without a stray character is one
// copy; one with strays is compacted 8 characters at a time (pext of the kept bytes).  dst needs
// 32 bytes of slack.
__attribute__((target("avx2,bmi2,popcnt"))) size_t compact_alphabet_avx2(const unsigned char* s, size_t& i, size_t end,
                                                                        unsigned char* dst, size_t want) {
    size_t got = 0;
    while (got + 32 <= want && i + 32 <= end) {
        const uint32_t bad = bad_mask32(s + i);
        if (!bad) {
            _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + got),
                                _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i)));
            got += 32;
        } else {
            for (int j = 0; j < 4; ++j) {
                const uint64_t keep = ~(bad >> (8 * j)) & 0xFFu;
                uint64_t w;
                std::memcpy(&w, s + i + 8 * j, 8);
                const uint64_t packed = _pext_u64(w, _pdep_u64(keep, 0x0101010101010101ull) * 0xFFu);
                std::memcpy(dst + got, &packed, 8);
                got += (size_t)__builtin_popcountll(keep);
            }
        }
        i += 32;
    }
    for (; got < want && i < end; ++i) {
        dst[got] = s[i];
        got += kT.v[s[i]] >= 0;
    }
    return got;
}

size_t compact_alphabet(const unsigned char* s, size_t& i, size_t end, unsigned char* dst, size_t want) {
    if (have_avx2_bmi2()) return compact_alphabet_avx2(s, i, end, dst, want);
    size_t got = 0;
    for (; got < want && i < end; ++i) {
        dst[got] = s[i];
        got += kT.v[s[i]] >= 0;
    }
    return got;
}

bool decode_clean(const unsigned char* in, size_t n4, uint8_t* out) {
    return have_avx2() ? decode_clean_avx2(in, n4, out) : decode_clean_scalar(in, n4, out);
}

bool all_alphabet(const unsigned char* in, size_t n) {
    if (have_avx2()) return all_alphabet_avx2(in, n);
    for (size_t i = 0; i < n; ++i)
        if (kT.v[in[i]] < 0) return false;
    return true;
}

// Populate the pages of a fresh output range in one call (MADV_POPULATE_WRITE, Linux 5.14+)
// instead of one page fault per 4 KiB during the decode; best effort (older kernels: no-op).
void populate(uint8_t* p, size_t n) {
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
    if (!p || n < (1u << 20)) return;
    static const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = ((uintptr_t)p + page - 1) & ~(page - 1), b = ((uintptr_t)p + n) & ~(page - 1);
    if (b > a) (void)madvise((void*)a, b - a, MADV_POPULATE_WRITE);
}

// The 2 MiB-aligned interior of a big fresh output on transparent huge pages (one fault per 2 MiB
// instead of 512): a 47 MB diff decodes in 7-9 ms instead of 11-12 (profiles/r02ad/).  One call
// over the whole output on the caller's thread, before the threads populate their parts (the
// hint changes the mapping's flags: one writer, not one per thread).
void hugepage_hint(uint8_t* p, size_t n) {
    if (!p || n < (4u << 20)) return;
    const uintptr_t h = (uintptr_t)2 << 20, ha = ((uintptr_t)p + h - 1) & ~(h - 1), hb = ((uintptr_t)p + n) & ~(h - 1);
    if (hb > ha) (void)madvise((void*)ha, hb - ha, MADV_HUGEPAGE);
}

// A persistent pool (thread creation cost ~1 ms per decode at 16 threads x 2 passes): run(t, f)
// calls f(k) for k in [0, t), k = 0 on the caller's thread.  One decode at a time per pool.
class Pool {
  public:
    void run(int t, const std::function<void(int)>& f) {
        std::lock_guard<std::mutex> one(busy_);
        if (t <= 1) { f(0); return; }
        grow(t - 1);
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &f;
            want_ = t - 1;
            pending_ = t - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }

  private:
    void grow(int n) {
        while ((int)workers_.size() < n) {
            const int id = (int)workers_.size() + 1;
            workers_.emplace_back([this, id] { loop(id); });
        }
    }
    void loop(int id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* fn = nullptr;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                if (id > want_) continue;  // not needed for this job
                fn = fn_;
            }
            (*fn)(id);
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::mutex busy_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* fn_ = nullptr;
    int want_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

Pool& pool() {
    static Pool* p = new Pool();  // never destroyed: worker threads must not be joined at exit
    return *p;
}

template <class F>
void parallel(int t, F&& f) {  // f(k) for k in [0, t), k = 0 on the calling thread
    const std::function<void(int)> fn = f;
    pool().run(t, fn);
}

}  // namespace

namespace {
// The fast path: every character before the first '=' in the alphabet.  Returns PGH_OK (decoded,
// *written set), PGH_E_PARSE (clean text, bad padding) or PGH_E_STATE (not clean, or more than
// cap bytes: nothing usable written).
int decode_fast(const unsigned char* s, size_t n, size_t fe, uint8_t* out, size_t cap, size_t* written, int t) {
    const size_t n4f = fe / 4;
    Machine m;
    std::vector<uint8_t> tail;
    m.feed(s + 4 * n4f, n - 4 * n4f, &tail);  // the last 0-3 prefix characters, then from '='
    if (!all_alphabet(s + 4 * n4f, fe - 4 * n4f)) return PGH_E_STATE;
    const bool padded = m.done || m.quad_pos == 0;
    const size_t need = n4f * 3 + tail.size();
    if (padded && out && need > cap) return PGH_E_STATE;
    const int tf = n4f < (1u << 16) ? 1 : t;
    const size_t pq = (n4f + tf - 1) / tf;
    std::atomic<bool> clean{true};
    if (out && padded) hugepage_hint(out, 3 * n4f);
    parallel(tf, [&](int k) {
        const size_t g0 = std::min(n4f, pq * k), g1 = std::min(n4f, g0 + pq);
        const bool dec = out && padded;
        if (dec) populate(out + 3 * g0, 3 * (g1 - g0));  // this thread's part of the fresh output
        const bool ok = dec ? decode_clean(s + 4 * g0, g1 - g0, out + 3 * g0) : all_alphabet(s + 4 * g0, 4 * (g1 - g0));
        if (!ok) clean.store(false, std::memory_order_relaxed);
    });
    if (!clean.load()) return PGH_E_STATE;
    if (!padded) return PGH_E_PARSE;  // a clean prefix: the machine's verdict is final
    if (out && !tail.empty()) std::memcpy(out + 3 * n4f, tail.data(), tail.size());
    *written = need;
    return PGH_OK;
}

int threads_for(size_t n, int threads) {
    const int t = threads > 0 ? threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    return n < (1u << 18) ? 1 : t;
}

// Where the fast path takes the first '=' to be: the first one in the last 4 KiB of the text (a
// client's base64 ends in its padding), else n.  An earlier '=' sits inside the prefix the fast path
// decodes, whose per-thread alphabet check then fails (PGH_E_STATE: the general route decides) --
// so no single-threaded memchr over the whole 62 MB text (twice per report: size, then decode).
size_t first_eq(const unsigned char* s, size_t n) {
    const size_t from = n > 4096 ? n - 4096 : 0;
    const void* eq = n ? std::memchr(s + from, '=', n - from) : nullptr;
    return eq ? (size_t)((const unsigned char*)eq - s) : n;
}

}  // namespace

extern "C" {

// Decoded size upper bound for an input of n characters.
size_t pgh_b64_decoded_cap(size_t n) { return n / 4 * 3 + 3; }

// Decoded size of `in` IF every character before its first '=' is in the alphabet (not checked:
// O(characters from the last whole quad of that prefix on)).  PGH_E_PARSE when that tail does not
// decode cleanly -- the caller then takes the general route (pgh_b64_decode with out == NULL).
int pgh_b64_clean_size(const char* in, size_t n, size_t* size) {
    if ((!in && n) || !size) return PGH_E_ARG;
    const unsigned char* s = (const unsigned char*)in;
    const size_t fe = first_eq(s, n);
    const size_t n4f = fe / 4;
    Machine m;
    std::vector<uint8_t> tail;
    m.feed(s + 4 * n4f, n - 4 * n4f, &tail);
    if (!m.done && m.quad_pos != 0) return PGH_E_PARSE;
    *size = n4f * 3 + tail.size();
    return PGH_OK;
}


// One pass for a clean string: `out` holds cap bytes (pgh_b64_clean_size's value); PGH_E_STATE
// when the text is not all alphabet before its first '=' (or decodes to more than cap): then take
// the general route, pgh_b64_decode.
int pgh_b64_decode_clean(const char* in, size_t n, uint8_t* out, size_t cap, size_t* written, int threads) {
    if ((!in && n) || !written || !out) return PGH_E_ARG;
    const unsigned char* s = (const unsigned char*)in;
    return decode_fast(s, n, first_eq(s, n), out, cap, written, threads_for(n, threads));
}

// Decode `in` (n chars) into `out` (capacity >= pgh_b64_decoded_cap(n)); *written = bytes.
// out == NULL: validate and size only.  threads <= 0 picks min(16, hardware threads).  Returns
// PGH_OK or PGH_E_PARSE (Python's "Incorrect padding" / "cannot be 1 more than a multiple of 4").
int pgh_b64_decode(const char* in, size_t n, uint8_t* out, size_t* written, int threads) {
    if ((!in && n) || !written) return PGH_E_ARG;
    const unsigned char* s = (const unsigned char*)in;
    const int t = threads_for(n, threads);
    {
        const int rc = decode_fast(s, n, first_eq(s, n), out, pgh_b64_decoded_cap(n), written, t);
        if (rc != PGH_E_STATE) return rc;  // clean text: decoded, or a padding error
    }
    // per chunk of the text: its first '=' and the alphabet characters before it; the first chunk
    // holding an '=' ends the machine's prefix [0, fe) (no serial scan of the whole text for it)
    const size_t per = (n + t - 1) / t;
    std::vector<size_t> good((size_t)t, 0), eqs((size_t)t, n);
    parallel(t, [&](int k) {
        const size_t a = std::min(n, per * k), b = std::min(n, a + per);
        const void* e = b > a ? std::memchr(s + a, '=', b - a) : nullptr;
        const size_t ek = e ? (size_t)((const unsigned char*)e - s) : b;
        eqs[(size_t)k] = e ? ek : n;
        good[(size_t)k] = count_alphabet(s, a, ek);
    });
    size_t fe = n;
    for (int k = 0; k < t; ++k) {
        if (fe < n) good[(size_t)k] = 0;  // after the prefix
        else fe = eqs[(size_t)k];
    }
    // at[k]: index, among the prefix's alphabet characters, of chunk k's first one
    std::vector<size_t> at((size_t)t + 1, 0);
    for (int k = 0; k < t; ++k) at[(size_t)k + 1] = at[(size_t)k] + good[(size_t)k];
    const size_t d = at[(size_t)t], n4 = d / 4;
    // the machine runs over the prefix's last d % 4 alphabet characters, then from the first '='
    unsigned char lead[3];
    size_t nl = 0;
    for (size_t i = fe; i > 0 && nl < d % 4; --i)
        if (kT.v[s[i - 1]] >= 0) lead[nl++] = s[i - 1];
    std::reverse(lead, lead + nl);
    Machine m;
    std::vector<uint8_t> tail;
    m.feed(lead, nl, &tail);
    m.feed(s + fe, n - fe, &tail);
    if (!m.done && m.quad_pos != 0) return PGH_E_PARSE;
    *written = n4 * 3 + tail.size();
    if (!out) return PGH_OK;
    if (d == fe) {  // clean prefix: whole quads straight from the input
        const int td = n4 < (1u << 16) ? 1 : t;
        const size_t pq = (n4 + td - 1) / td;
        parallel(td, [&](int k) {
            const size_t g0 = std::min(n4, pq * k), g1 = std::min(n4, g0 + pq);
            decode_groups(s + 4 * g0, g1 - g0, out + 3 * g0);
        });
    } else {  // skip what the machine skips: thread k decodes the quads whose FIRST character is in its chunk
        parallel(t, [&](int k) {
            size_t i = std::min(fe, per * k), c = at[(size_t)k];
            const size_t c_end = std::min(at[(size_t)k + 1], 4 * n4);
            while (c % 4 && c < c_end) c += kT.v[s[i++]] >= 0;  // finishes a quad begun in an earlier chunk
            // its quads' characters, compacted piece by piece into a local buffer and decoded as
            // clean text (the last quad may read past the chunk: never past fe)
            size_t need = c < c_end ? (c_end - c + 3) / 4 * 4 : 0;
            uint8_t* o = out + 3 * (c / 4);
            constexpr size_t B = 16384;
            alignas(32) unsigned char buf[B + 32];
            while (need) {
                const size_t got = compact_alphabet(s, i, fe, buf, std::min(need, B));
                if (got % 4 || !got) break;  // cannot happen: the prefix holds 4 * n4 alphabet characters
                decode_clean(buf, got / 4, o);
                o += got / 4 * 3;
                need -= got;
            }
        });
    }
    if (!tail.empty()) std::memcpy(out + 3 * n4, tail.data(), tail.size());
    return PGH_OK;
}


}  // extern "C"
