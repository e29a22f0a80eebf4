// Host-only fuzz of the untrusted-input parsers (client State bytes, base64 diff text) under
// AddressSanitizer + UndefinedBehaviorSanitizer.  Built and run by tests/test_native_sanitizers.py
// with g++ (no HIP): pgh_state.cpp and pgh_b64.cpp need only include/pgh_api.h.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "pgh_api.h"

static void put_varint(std::vector<uint8_t>& b, uint64_t v) {
    while (v >= 0x80) { b.push_back((uint8_t)(v | 0x80)); v >>= 7; }
    b.push_back((uint8_t)v);
}
static void put_field(std::vector<uint8_t>& b, uint32_t f, const std::vector<uint8_t>& payload) {
    put_varint(b, (f << 3) | 2);
    put_varint(b, payload.size());
    b.insert(b.end(), payload.begin(), payload.end());
}

// A valid State (restated schema: tensors=2 -> torch_tensor=1 -> contents_data=4 -> shape=1,
// dtype=2, contents_float32=12) with `t` tensors of random sizes.
static std::vector<uint8_t> make_state(std::mt19937_64& rng, int t) {
    std::vector<uint8_t> st;
    for (int k = 0; k < t; ++k) {
        const int n = (int)(rng() % 40);
        std::vector<uint8_t> dims, size, td, tt, stt, payload(4 * (size_t)n, 0x3f);
        put_varint(dims, (uint64_t)n);
        put_field(size, 1, dims);
        put_field(td, 1, size);
        put_field(td, 2, std::vector<uint8_t>{'f', 'l', 'o', 'a', 't', '3', '2'});
        if (n) put_field(td, 12, payload);
        put_field(tt, 4, td);
        put_field(stt, 1, tt);
        put_field(st, 2, stt);
    }
    return st;
}

// A valid share State: every tensor a packed-varint contents_int64 payload (field 10).
static std::vector<uint8_t> make_share_state(std::mt19937_64& rng, int t) {
    std::vector<uint8_t> st;
    for (int k = 0; k < t; ++k) {
        const int n = (int)(rng() % 200);
        std::vector<uint8_t> dims, size, td, tt, stt, payload;
        for (int i = 0; i < n; ++i) put_varint(payload, rng() >> (rng() % 64));
        put_varint(dims, (uint64_t)n);
        put_field(size, 1, dims);
        put_field(td, 1, size);
        put_field(td, 2, std::vector<uint8_t>{'i', 'n', 't', '6', '4'});
        if (n) put_field(td, 10, payload);
        put_field(tt, 4, td);
        put_field(stt, 1, tt);
        put_field(st, 2, stt);
    }
    return st;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(12345);
    int parsed = 0, rejected = 0;
    for (int it = 0; it < iters; ++it) {
        std::vector<uint8_t> pb = make_state(rng, 1 + (int)(rng() % 5));
        const int muts = (int)(rng() % 6);
        for (int m = 0; m < muts && !pb.empty(); ++m) {
            const size_t i = rng() % pb.size();
            switch (rng() % 4) {
            case 0: pb[i] = (uint8_t)rng(); break;
            case 1: pb.resize(i); break;  // truncate
            case 2: pb.insert(pb.begin() + (long)i, (uint8_t)rng()); break;
            default: pb[i] ^= 0x80; break;  // flip varint continuation
            }
        }
        // exact-size heap copy so ASan sees any read past the end
        uint8_t* buf = new uint8_t[pb.size() ? pb.size() : 1];
        if (!pb.empty()) std::memcpy(buf, pb.data(), pb.size());
        int nt = 0;
        int64_t offs[8], cnts[8];
        const int rc = pgh_state_scan(buf, pb.size(), 8, offs, cnts, &nt);
        if (rc == PGH_OK) {
            ++parsed;
            int64_t total = 0;
            for (int k = 0; k < nt && k < 8; ++k) {
                if (offs[k] < 0 || (size_t)(offs[k] + 4 * cnts[k]) > pb.size()) { std::printf("span out of range\n"); return 2; }
                total += cnts[k];
            }
            if (nt <= 8) {
                std::vector<float> vals((size_t)total + 1, 1.0f);
                std::vector<uint8_t> out(pb.size() ? pb.size() : 1, 0xCD);  // poison: every byte must be written
                if (pgh_state_patch(buf, pb.size(), vals.data(), total, out.data()) != PGH_OK) { std::printf("patch failed\n"); return 3; }
                std::vector<uint8_t> want(pb.begin(), pb.end());  // template, then payloads in span order
                int64_t vo = 0;
                for (int k = 0; k < nt; ++k) {
                    std::memcpy(want.data() + offs[k], vals.data() + vo, 4 * (size_t)cnts[k]);
                    vo += cnts[k];
                }
                if (!pb.empty() && std::memcmp(want.data(), out.data(), pb.size()) != 0) { std::printf("patch bytes differ\n"); return 5; }
            }
        } else {
            ++rejected;
        }
        delete[] buf;
        // int64 share States: the walker plus the varint count / overlong pass
        std::vector<uint8_t> sh = make_share_state(rng, 1 + (int)(rng() % 4));
        const int smuts = (int)(rng() % 4);
        for (int m = 0; m < smuts && !sh.empty(); ++m) {
            const size_t i = rng() % sh.size();
            switch (rng() % 3) {
            case 0: sh[i] |= 0x80; break;   // lengthen a varint
            case 1: sh.resize(i); break;
            default: sh[i] = (uint8_t)rng(); break;
            }
        }
        uint8_t* sbuf = new uint8_t[sh.size() ? sh.size() : 1];
        if (!sh.empty()) std::memcpy(sbuf, sh.data(), sh.size());
        int64_t so[8], sn[8], sc[8];
        nt = 0;
        if (pgh_state_scan_i64(sbuf, sh.size(), 8, so, sn, sc, &nt) == PGH_OK) {
            ++parsed;
            for (int k = 0; k < nt && k < 8; ++k) {
                if (so[k] < 0 || (size_t)(so[k] + sn[k]) > sh.size() || sc[k] > sn[k]) { std::printf("share span out of range\n"); return 6; }
                int64_t term = 0;  // the count is the number of terminator bytes
                for (int64_t i = 0; i < sn[k]; ++i) term += !(sbuf[so[k] + i] & 0x80);
                if (term != sc[k]) { std::printf("share count mismatch\n"); return 7; }
            }
        } else {
            ++rejected;
        }
        delete[] sbuf;
        // base64 text with random junk
        std::string s;
        const int len = (int)(rng() % 64);
        const char* alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/= \n*";
        for (int k = 0; k < len; ++k) s.push_back(alpha[rng() % 67]);
        char* txt = new char[s.size() ? s.size() : 1];
        std::memcpy(txt, s.data(), s.size());
        size_t w = 0;
        if (pgh_b64_decode(txt, s.size(), nullptr, &w, 1) == PGH_OK) {
            std::vector<uint8_t> out(w ? w : 1);
            size_t w2 = 0;
            if (pgh_b64_decode(txt, s.size(), out.data(), &w2, 1) != PGH_OK || w2 != w) { std::printf("b64 size mismatch\n"); return 4; }
        }
        delete[] txt;
        // long, mostly clean base64 (the AVX2 fast path: 32-character blocks) with rare junk, decoded
        // through pgh_b64_clean_size + pgh_b64_decode_clean into an exact-size heap buffer
        {
            const int blen = 32 + (int)(rng() % 400);
            std::string t;
            for (int k = 0; k < blen; ++k) t.push_back(rng() % 97 == 0 ? alpha[rng() % 67] : alpha[rng() % 64]);
            char* bt = new char[t.size()];
            std::memcpy(bt, t.data(), t.size());
            size_t want = 0, w3 = 0;
            if (pgh_b64_clean_size(bt, t.size(), &want) == PGH_OK) {
                uint8_t* o = new uint8_t[want ? want : 1];
                const int rc3 = pgh_b64_decode_clean(bt, t.size(), o, want, &w3, 1 + (int)(rng() % 3));
                if (rc3 == PGH_OK && w3 != want) { std::printf("b64 clean size mismatch\n"); return 8; }
                delete[] o;
            }
            size_t w4 = 0;
            if (pgh_b64_decode(bt, t.size(), nullptr, &w4, 2) == PGH_OK) {
                std::vector<uint8_t> o(pgh_b64_decoded_cap(t.size()));
                size_t w5 = 0;
                if (pgh_b64_decode(bt, t.size(), o.data(), &w5, 2) != PGH_OK || w5 != w4) { std::printf("b64 long mismatch\n"); return 9; }
            }
            delete[] bt;
        }
        // fresh checkpoint framing of a (mutated) template into an exact-size buffer
        {
            std::vector<uint8_t> tp = make_state(rng, 1 + (int)(rng() % 4));
            if (rng() % 2 && !tp.empty()) tp[rng() % tp.size()] = (uint8_t)rng();
            uint8_t* tb = new uint8_t[tp.size() ? tp.size() : 1];
            if (!tp.empty()) std::memcpy(tb, tp.data(), tp.size());
            int ntt = 0;
            if (pgh_state_scan(tb, tp.size(), 0, nullptr, nullptr, &ntt) == PGH_OK && ntt <= 8) {
                int64_t ids[16];
                for (int k = 0; k < 2 * ntt; ++k) ids[k] = (int64_t)(rng() % 100000000000ull);
                size_t need = 0, need2 = 0;
                if (pgh_state_fresh(tb, tp.size(), ids, 2 * ntt, nullptr, 0, &need) == PGH_OK) {
                    uint8_t* fo = new uint8_t[need ? need : 1];
                    if (pgh_state_fresh(tb, tp.size(), ids, 2 * ntt, fo, need, &need2) != PGH_OK || need2 != need) {
                        std::printf("fresh framing failed\n");
                        return 10;
                    }
                    int nf = 0;  // the fresh framing scans back with the same tensor count
                    if (pgh_state_scan(fo, need, 0, nullptr, nullptr, &nf) != PGH_OK || nf != ntt) {
                        std::printf("fresh framing does not scan back\n");
                        return 11;
                    }
                    delete[] fo;
                }
            }
            delete[] tb;
        }
    }
    std::printf("ok parsed=%d rejected=%d\n", parsed, rejected);
    return 0;
}
