// Pointer-chase throughput of wave-uniform loads: scalar (s_load via the
// scalar cache) vs vector (global_load, uniform address, readfirstlane), as a
// function of resident waves per CU and of independent chains per wave.
// Table: 96 MB of u32 "next line" indices (random permutation of 64-B lines).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

typedef __attribute__((address_space(4))) const unsigned cu32_t;

template <int CHAINS, bool SCALAR>
__global__ void __launch_bounds__(256) chase(const unsigned *tab, unsigned steps, unsigned *out) {
    const unsigned wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    unsigned idx[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) idx[c] = (wave * 7919u + c * 104729u) & ((96u << 20) / 64 - 1);
    for (unsigned s = 0; s < steps; ++s) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (SCALAR) {
                idx[c] = ((cu32_t *)(const void *)tab)[idx[c] * 16];
            } else {
                idx[c] = __builtin_amdgcn_readfirstlane(tab[idx[c] * 16]);
            }
        }
    }
    unsigned acc = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc += idx[c];
    if ((threadIdx.x & 63) == 0) out[wave] = acc;
}

template <int CHAINS, bool SCALAR>
double run(const unsigned *tab, unsigned *out, int blocks, unsigned steps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((chase<CHAINS, SCALAR>), dim3(blocks), dim3(256), 0, 0, tab, 64u, out);
    hipEventRecord(a);
    hipLaunchKernelGGL((chase<CHAINS, SCALAR>), dim3(blocks), dim3(256), 0, 0, tab, steps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    const double loads = (double)blocks * 4 * steps * CHAINS;
    return loads / (ms * 1e-3) / 256.0 / 1e6;   // M loads/s per CU
}

int main() {
    const size_t lines = (96u << 20) / 64;
    std::vector<unsigned> perm(lines);
    for (size_t i = 0; i < lines; ++i) perm[i] = (unsigned)i;
    std::mt19937 rng(1);
    std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<unsigned> tab(lines * 16, 0);
    for (size_t i = 0; i < lines; ++i) tab[perm[i] * 16] = perm[(i + 1) % lines];
    unsigned *dt, *dout;
    hipMalloc(&dt, tab.size() * 4);
    hipMemcpy(dt, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&dout, 1 << 24);
    const unsigned steps = 2000;
    printf("waves/CU  scalar1  scalar2  scalar4  vector1  vector2  vector4   (M loads/s per CU)\n");
    for (int bpc : {1, 2, 4, 7, 8}) {
        const int blocks = 256 * bpc;
        printf("%8d %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f\n", bpc * 4,
               run<1, true>(dt, dout, blocks, steps), run<2, true>(dt, dout, blocks, steps),
               run<4, true>(dt, dout, blocks, steps), run<1, false>(dt, dout, blocks, steps),
               run<2, false>(dt, dout, blocks, steps), run<4, false>(dt, dout, blocks, steps));
    }
    return 0;
}
