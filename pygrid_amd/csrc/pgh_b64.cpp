// Standard-alphabet base64 decode for the report path (host only).
//
// Reference: fl_events.report decodes every client diff with
// `base64.b64decode(data.get(CYCLE.DIFF, None).encode())` (apps/node/src/app/main/events/
// model_centric/fl_events.py:257) -- O(diff bytes) per request, 47 MB per ResNet-18 diff.  Every
// 4-character group decodes independently, so the input is split into group-aligned ranges
// decoded by parallel threads.  Semantics follow Python's default (validate=False): characters
// outside the alphabet (whitespace, newlines) are discarded before decoding, '=' padding ends
// the data; a group count that is not a multiple of 4 after that is an error ("Incorrect padding").
#include <algorithm>
#include <cstdint>
#include <cstring>
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

// Decode `n4` complete groups of clean input (no padding) into out; returns bytes written.
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

}  // namespace

extern "C" {

// Decoded size upper bound for an input of n characters.
size_t pgh_b64_decoded_cap(size_t n) { return n / 4 * 3 + 3; }

// Decode `in` (n chars) into `out` (capacity >= pgh_b64_decoded_cap(n)); *written = bytes.
// out == NULL: validate only and return the exact decoded size in *written.
// threads <= 0 picks min(16, hardware threads).  Returns PGH_OK or PGH_E_PARSE (Python's
// "Incorrect padding" / "cannot be 1 more than a multiple of 4").
int pgh_b64_decode(const char* in, size_t n, uint8_t* out, size_t* written, int threads) {
    if ((!in && n) || !written) return PGH_E_ARG;  // out == NULL: validate and size only
    const unsigned char* s = (const unsigned char*)in;
    int t = threads > 0 ? threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (n < (1u << 18)) t = 1;
    // data ends at the first '='; everything before it must be alphabet for the fast path
    const void* eq = n ? std::memchr(s, '=', n) : nullptr;
    const size_t fe = eq ? (size_t)((const unsigned char*)eq - s) : n;
    std::vector<char> bad((size_t)t, 0);
    {
        const size_t per = (fe + t - 1) / t;
        std::vector<std::thread> th;
        auto scan = [&](int k) {
            const size_t a = per * k, b = std::min(fe, a + per);
            for (size_t i = a; i < b; ++i)
                if (kT.v[s[i]] < 0) { bad[(size_t)k] = 1; return; }
        };
        for (int k = 1; k < t; ++k) th.emplace_back(scan, k);
        scan(0);
        for (auto& x : th) x.join();
    }
    bool clean = true;
    for (char b : bad) clean = clean && !b;
    std::vector<unsigned char> filtered;
    size_t d = fe;
    if (!clean) {  // non-validating decode: drop characters outside the alphabet
        filtered.reserve(fe);
        for (size_t k = 0; k < fe; ++k)
            if (kT.v[s[k]] >= 0) filtered.push_back(s[k]);
        d = filtered.size();
    }
    // padding: '=' characters from the first one on (other non-alphabet characters skipped)
    size_t pads = 0;
    for (size_t k = fe; k < n; ++k) {
        if (s[k] == '=') ++pads;
        else if (kT.v[s[k]] >= 0) break;
    }
    const unsigned char* data = clean ? s : filtered.data();
    const size_t rem = d % 4;
    if (rem == 1) return PGH_E_PARSE;
    if ((rem == 2 && pads < 2) || (rem == 3 && pads < 1)) return PGH_E_PARSE;
    const size_t n4 = d / 4;
    if (!out) {
        *written = n4 * 3 + (rem == 2 ? 1 : rem == 3 ? 2 : 0);
        return PGH_OK;
    }
    if (n4 < (1u << 16)) t = 1;
    const size_t per = (n4 + t - 1) / t;
    std::vector<std::thread> th;
    for (int k = 1; k < t; ++k) {
        const size_t g0 = per * k;
        if (g0 >= n4) break;
        const size_t g1 = std::min(n4, g0 + per);
        th.emplace_back([=] { decode_groups(data + 4 * g0, g1 - g0, out + 3 * g0); });
    }
    decode_groups(data, std::min(per, n4), out);
    for (auto& x : th) x.join();
    size_t w = n4 * 3;
    if (rem) {  // 2 or 3 trailing characters -> 1 or 2 bytes
        const unsigned char* r = data + 4 * n4;
        uint32_t x = ((uint32_t)kT.v[r[0]] << 18) | ((uint32_t)kT.v[r[1]] << 12);
        if (rem == 3) x |= (uint32_t)kT.v[r[2]] << 6;
        out[w++] = (uint8_t)(x >> 16);
        if (rem == 3) out[w++] = (uint8_t)(x >> 8);
    }
    *written = w;
    return PGH_OK;
}

}  // extern "C"
