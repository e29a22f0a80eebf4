/* CPU check of the iterative fold's division shortcut (pgh_kernels.hip, fold<MODE_ITERATIVE>):
 *
 *     t / (float)y  ==  (float)((double)t * (1.0 / (double)y))     for integer 2 <= y <= 2^24,
 *
 * whenever the product is 0, inf, NaN or at least 2^-125 in magnitude (the kernel divides for
 * real below that).  Why it holds: the double product is within ~2^-52 (relative) of t / y, while
 * t / y, if not exactly an f32 rounding midpoint, is at least ~2^-49 away from one in the normal
 * range -- and it is never exactly a midpoint there (a 25-bit odd significand cannot divide a
 * 24-bit one).  Among subnormal quotients exact ties DO occur and the product alone can round
 * them the wrong way (147 * 2^-149 / 98: tie -> 2^-148, product -> 2^-149), hence the fallback.
 * Checked here on random and adversarial operands against IEEE float division.
 *
 *   cc -O2 -ffp-contract=off -o recip_div_check recip_div_check.c && ./recip_div_check [samples]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x243F6A8885A308D3ull;
static uint64_t rnd(void) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static long checked = 0, fallback = 0;
static int check(float t, uint32_t y) {
    volatile float yf = (float)y;
    const float want = t / yf;
    const double r = 1.0 / (double)y;
    const double q = (double)t * r;
    float got = (float)q;
    if (fabs(q) < 0x1p-125 && q != 0.0) { got = t / yf; ++fallback; }
    ++checked;
    if (isnan(want) && isnan(got)) return 0;
    if (u_of(want) != u_of(got)) {
        printf("MISMATCH t=%a (0x%08x) y=%u want=%a got=%a\n", t, u_of(t), y, want, got);
        return 1;
    }
    return 0;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 10000000;
    int bad = 0;
    for (long i = 0; i < n && !bad; ++i) {
        const uint64_t a = rnd();
        /* y: small, around powers of two, or anywhere up to 2^24 */
        uint32_t y;
        switch (a & 3) {
        case 0: y = 2 + (uint32_t)((a >> 8) % 1000); break;
        case 1: { const int e = 1 + (int)((a >> 8) % 24); y = (1u << e) + (uint32_t)((int)((a >> 16) % 5) - 2); break; }
        default: y = 2 + (uint32_t)((a >> 8) % ((1u << 24) - 1)); break;
        }
        if (y < 2) y = 2;
        if (y > (1u << 24)) y = 1u << 24;
        /* t: any bit pattern, or t = (near-)multiple of y times a value near a midpoint */
        float t;
        if ((a >> 60) & 1) {
            t = f_of((uint32_t)(a >> 32));
        } else {
            const float m = f_of((uint32_t)rnd() & 0x7fffffffu | 0x00800000u);  /* normal */
            t = m * (float)y;                                               /* rounds: near-exact quotient */
            uint32_t u = u_of(t);
            u += (uint32_t)((int)((a >> 40) % 7) - 3);
            t = f_of(u);
        }
        bad |= check(t, y);
        bad |= check(-t, y);
    }
    /* exact subnormal ties t / y = odd * 2^-150 (y even, t = odd * y / 2 * 2^-149) */
    for (uint32_t y = 2; y < 4096 && !bad; y += 2)
        for (uint32_t m = 1; (uint64_t)m * (y / 2) < (1u << 23) && !bad; m += 2 + 2 * (y > 512) * 30)
            bad |= check(f_of(m * (y / 2)), y);
    /* all subnormal and smallest-normal t against a few y */
    for (uint32_t u = 0; u < 0x01000000u && !bad; u += 37)
        for (uint32_t y = 2; y < 40 && !bad; y += 3) bad |= check(f_of(u), y);
    printf("%s checked=%ld fallback=%ld\n", bad ? "FAIL" : "ok", checked, fallback);
    return bad;
}
