// Prints the distinct (XCC_ID, HW_ID.se/sh/cu) keys seen by a full grid:
// checks the CU-key layout the render kernel's per-CU tile queues assume.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <set>
#include <vector>

__global__ void k(unsigned *o) {
    unsigned x, h;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
    if (threadIdx.x == 0) { o[2 * blockIdx.x] = x; o[2 * blockIdx.x + 1] = h; }
}

int main() {
    const int nb = 256 * 16;
    unsigned *d;
    (void)hipMalloc(&d, nb * 8);
    hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, d);
    std::vector<unsigned> h(2 * nb);
    (void)hipMemcpy(h.data(), d, nb * 8, hipMemcpyDeviceToHost);
    std::set<unsigned> keys, xcc, se, sh, cu;
    for (int i = 0; i < nb; ++i) {
        unsigned x = h[2 * i] & 0xf, w = h[2 * i + 1];
        unsigned c = (w >> 8) & 0xf, s = (w >> 12) & 1, e = (w >> 13) & 0x7;
        keys.insert((x << 7) | (e << 5) | (s << 4) | c);
        xcc.insert(x); se.insert(e); sh.insert(s); cu.insert(c);
        if (i < 8) printf("block %d xcc %u hwid 0x%08x se %u sh %u cu %u\n", i, x, w, e, s, c);
    }
    printf("distinct keys %zu xcc %zu se %zu sh %zu cu %zu\n", keys.size(), xcc.size(), se.size(),
           sh.size(), cu.size());
    return 0;
}
