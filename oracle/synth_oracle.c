/*
 * synth_oracle.c — CPU twin of the synthetic corpus generator
 * (syzkaller_amd/csrc/synth.hip).  SURVEY §8d spec, made integer-exact so
 * host and device regenerate bit-identical corpora:
 *   universe  U[k] = 0x81000000 + 16k + (h(k) & 15), k < 2^S  (S = log2_space)
 *   length    L_i  = clamp(round(mean + sigma * z_i), 1, 65535), z_i = Irwin-Hall(12) - 6
 *                    (integer stand-in for the Box-Muller normal of §8d)
 *   draw      k    = floor(2^S * u^3), u = x / 2^32, x = 32 hash bits  -> (x^3) >> (96 - S)
 *                    (every key < 2^S is reachable; S <= 32)
 *             (uniform variant: k = top S hash bits)
 *   x86 universe (mode bit 1): U[2m] = 0x81000000 + 16m + a, U[2m+1] = U[2m] + 5 + b,
 *                (a, b) = 2-bit fields of h(m): neighbours 5..14 B apart, kshift 2
 * TEST INFRASTRUCTURE ONLY.
 */
#include "oracle.h"

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint32_t orc_synth_universe_mode(uint64_t seed, uint32_t k, int mode) {
    if (mode & 2) { /* x86-like: pairs per 16-byte block, gaps 5..14 */
        uint64_t h = splitmix64(seed ^ 0xA0761D6478BD642Full ^ (uint64_t)(k >> 1));
        return 0x81000000u + 16u * (k >> 1) + (uint32_t)(h & 3u) +
               (k & 1u) * (5u + (uint32_t)((h >> 2) & 3u));
    }
    uint64_t h = splitmix64(seed ^ 0xA0761D6478BD642Full ^ (uint64_t)k);
    return 0x81000000u + 16u * k + (uint32_t)(h & 15u);
}

uint32_t orc_synth_universe(uint64_t seed, uint32_t k) { return orc_synth_universe_mode(seed, k, 0); }

uint32_t orc_synth_len(uint64_t seed, uint64_t input, uint32_t mean, uint32_t sigma) {
    uint64_t base = splitmix64(seed ^ splitmix64(input ^ 0x5851F42D4C957F2Dull));
    int64_t sum = 0;
    for (int t = 0; t < 3; t++) {
        uint64_t h = splitmix64(base + (uint64_t)(t + 1) * 0x9E3779B97F4A7C15ull);
        sum += (int64_t)(h & 0xFFFF) + (int64_t)((h >> 16) & 0xFFFF) +
               (int64_t)((h >> 32) & 0xFFFF) + (int64_t)(h >> 48);
    }
    int64_t num = (int64_t)sigma * (sum - 6 * 65536) + 32768;
    int64_t off = num >= 0 ? num / 65536 : -((-num + 65535) / 65536); /* floor */
    int64_t L = (int64_t)mean + off;
    if (L < 1) L = 1;
    if (L > 65535) L = 65535;
    return (uint32_t)L;
}

/* mode bit 0: uniform draws; bit 1: the x86-like universe */
void orc_synth_input(uint64_t seed, uint64_t input, uint32_t len, uint32_t log2_space,
                     int mode, uint32_t *out) {
    const int uniform = mode & 1;
    uint64_t base = splitmix64(seed ^ splitmix64(input + 0x632BE59BD9B4E019ull));
    for (uint32_t j = 0; j < len; j++) {
        uint64_t h = splitmix64(base + (uint64_t)(j + 1) * 0x9E3779B97F4A7C15ull);
        uint32_t k;
        if (uniform) {
            k = (uint32_t)(h >> (64 - log2_space));
        } else {
            uint64_t x = h >> 32; /* 32 bits; x^3 < 2^96 */
            k = (uint32_t)((uint64_t)(((unsigned __int128)(x * x) * x) >> 64) >> (32 - log2_space));
        }
        out[j] = orc_synth_universe_mode(seed, k, mode);
    }
}

/* C5 (syz-fuzzer execute): the CallID of synthetic call record `input`,
 * uniform over [0, ncalls) (the multiply-high of a 32-bit hash: no modulo). */
int32_t orc_synth_callid(uint64_t seed, uint64_t input, uint32_t ncalls) {
    uint64_t h = splitmix64(seed ^ splitmix64(input ^ 0xC2B2AE3D27D4EB4Full));
    return (int32_t)(((h >> 32) * (uint64_t)ncalls) >> 32);
}
