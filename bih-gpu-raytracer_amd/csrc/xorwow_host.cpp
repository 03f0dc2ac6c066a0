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

std::once_flag g_once;
std::vector<uint32_t> g_tables;   // [32 seq][160][5] ++ [64 step][160][5]

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

}  // namespace bih
