// xorwow_host.cpp -- cuRAND-compatible XORWOW seeding and GF(2) jump tables.
//
// The reference seeds one curandState per pixel with
// curand_init(1984, pixel_index, 0) (src/CUDAKernels.cu:450-459) and draws
// with curand_uniform (:414-415).  cuRAND is not vendored by the reference;
// its XORWOW is restated here from cuRAND's public header semantics:
//   seed salt   s0 = lo32(seed) ^ 0xaad26b49, s1 = hi32(seed) ^ 0xf7dcefdd,
//               t0 = 1099087573*s0, t1 = 2591861531*s1,
//               v = {123456789+t0, 362436069^t0, 521288629+t1, 88675123^t1,
//                    5783321+t0}, d = 6615241+t1+t0
//   subsequence i starts 2^67*i steps in (d unchanged: 2^67*362437 = 0 mod 2^32)
// The 160-bit linear part v is advanced with precomputed powers of the
// step matrix M over GF(2):  seq[k] = M^(2^(67+k)), step[k] = M^(2^k).
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "bih_internal.h"

namespace bih {
namespace {

struct Gf2 {
    uint32_t c[160][5];   // column b = image of unit vector b
};

void step_lin(uint32_t v[5]) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1];
    v[1] = v[2];
    v[2] = v[3];
    v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}

void apply(const Gf2 &A, uint32_t x[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < 160; ++b)
        if ((x[b >> 5] >> (b & 31)) & 1u)
            for (int w = 0; w < 5; ++w) r[w] ^= A.c[b][w];
    memcpy(x, r, sizeof r);
}

void square(const Gf2 &A, Gf2 &out) {
    for (int b = 0; b < 160; ++b) {
        uint32_t x[5];
        memcpy(x, A.c[b], sizeof x);
        apply(A, x);
        memcpy(out.c[b], x, sizeof x);
    }
}

// C = A o B (all tables are powers of one matrix, so they commute)
void mul(const Gf2 &A, const Gf2 &B, Gf2 &C) {
    for (int b = 0; b < 160; ++b) {
        uint32_t x[5];
        memcpy(x, B.c[b], sizeof x);
        apply(A, x);
        memcpy(C.c[b], x, sizeof x);
    }
}

std::once_flag g_once, g_once_dev;
std::vector<uint32_t> g_tables;   // [32 seq][160][5] ++ [64 step][160][5]
std::vector<uint32_t> g_dev;      // device init tables, see xorwow_init_tables_host

void build_tables() {
    std::vector<Gf2> step(64), seq(32);
    for (int b = 0; b < 160; ++b) {
        uint32_t x[5] = {0, 0, 0, 0, 0};
        x[b >> 5] = 1u << (b & 31);
        step_lin(x);
        memcpy(step[0].c[b], x, sizeof x);
    }
    for (int k = 1; k < 64; ++k) square(step[k - 1], step[k]);
    Gf2 t = step[63], u;
    for (int k = 0; k < 4; ++k) {   // M^(2^63) -> M^(2^67)
        square(t, u);
        t = u;
    }
    seq[0] = t;
    for (int k = 1; k < 32; ++k) square(seq[k - 1], seq[k]);
    g_tables.resize((32 + 64) * 160 * 5);
    uint32_t *p = g_tables.data();
    for (int k = 0; k < 32; ++k, p += 800) memcpy(p, seq[k].c, 800 * 4);
    for (int k = 0; k < 64; ++k, p += 800) memcpy(p, step[k].c, 800 * 4);
}

}  // namespace

void xorwow_seed(uint64_t seed, uint32_t v[5], uint32_t *d) {
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    *d = 6615241u + t1 + t0;
    v[0] = 123456789u + t0;
    v[1] = 362436069u ^ t0;
    v[2] = 521288629u + t1;
    v[3] = 88675123u ^ t1;
    v[4] = 5783321u + t0;
}

const uint32_t *xorwow_tables_host() {
    std::call_once(g_once, build_tables);
    return g_tables.data();
}

void xorwow_skip(uint32_t v[5], uint64_t skip) {
    const uint32_t *step = xorwow_tables_host() + 32 * 800;
    for (int k = 0; skip && k < 64; ++k, skip >>= 1)
        if (skip & 1) {
            Gf2 m;
            memcpy(m.c, step + k * 800, sizeof m.c);
            apply(m, v);
        }
}

// k_rng_init's tables: jump bytes [4][256][160][5], entry (k, b) = J^(b << 8k)
// with J = M^(2^67) (one subsequence), so a pixel's subsequence start is at
// most 4 matrix applies; then J and J^64 by 4-bit input groups [2][40][16][5]
// (entry (g, n) = XOR of the matrix's columns 4g + set bits of n), a lane's
// step to its next pixel from LDS; then the frame jumps [7][40][16][5].
static void build_init_tables() {
    const uint32_t *seqt = xorwow_tables_host();
    std::vector<Gf2> seq(32);
    for (int k = 0; k < 32; ++k) memcpy(seq[k].c, seqt + k * 800, 800 * 4);
    g_dev.assign(kRngInitWords, 0u);
    uint32_t *bytes = g_dev.data();
    Gf2 id{};
    for (int b = 0; b < 160; ++b) id.c[b][b >> 5] = 1u << (b & 31);
    std::vector<Gf2> lvl(256);
    for (int k = 0; k < 4; ++k) {
        lvl[0] = id;
        for (int b = 1; b < 256; ++b) mul(lvl[b & (b - 1)], seq[8 * k + __builtin_ctz(b)], lvl[b]);
        for (int b = 0; b < 256; ++b) memcpy(bytes + ((size_t)k * 256 + b) * 800, lvl[b].c, 800 * 4);
    }
    // nibble tables of J (k_rng_init's per-pixel step) and of J^64 (a lane's
    // step when the 64 lanes of a wave seed 64 consecutive pixels at a time)
    // ... and of M^(2^(7+l)), l = 0..6: k_rng_sync's jump of kStampJumpFrames
    // = 64 frames of 2 * 2^l draws at spp 2^l
    std::vector<Gf2> fj(7);
    const uint32_t *stept = seqt + 32 * 800;
    for (int l = 0; l < 7; ++l) memcpy(fj[l].c, stept + (7 + l) * 800, 800 * 4);
    const Gf2 *steps[9] = {&seq[0], &seq[6], &fj[0], &fj[1], &fj[2], &fj[3], &fj[4], &fj[5], &fj[6]};
    static_assert(kStampJumpFrames == 64, "the frame-jump tables are M^(2^(7+l))");
    for (int t = 0; t < 9; ++t) {
        uint32_t *nib = bytes + 4 * 256 * 800 + t * 40 * 16 * 5;
        for (int g = 0; g < 40; ++g)
            for (int n = 0; n < 16; ++n)
                for (int j = 0; j < 4; ++j)
                    if ((n >> j) & 1)
                        for (int w = 0; w < 5; ++w) nib[(g * 16 + n) * 5 + w] ^= steps[t]->c[4 * g + j][w];
    }
}

const uint32_t *xorwow_init_tables_host() {
    std::call_once(g_once_dev, build_init_tables);
    return g_dev.data();
}

}  // namespace bih
