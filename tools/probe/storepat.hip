// Write-pattern probe 2 (diagnostic, not part of the product): env blocks of B bytes written by
// whole waves, XCD-local (workgroup b on XCD b % 8 writes into the x-th eighth of the buffer), with
// NW writer waves per workgroup (one workgroup per CU) and K waves sharing one block (piece j of
// 1 KB by wave j % K of the block's group).  hipcc --offload-arch=gfx950 -O3 -o storepat storepat.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// block b of the XCD is written by wave group g = b % groups (K waves), pieces k = lane + 64 i
template <int K, int THR>
__global__ void __launch_bounds__(1024) k_pat(v4u* o, int nblk, int per16, int nw) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
    const int bx = nblk / 8;
    v4u* base = o + (size_t)x * bx * per16;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w >= nw) return;
    const int groups_per_wg = nw / K, gw = w / K, kk = w % K;
    for (int b = j * groups_per_wg + gw; b < bx; b += nj * groups_per_wg) {
        v4u* p = base + (size_t)b * per16;
        for (int k = (kk * 64) + lane; k < per16; k += 64 * K) {
            p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
            if (THR >= 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(THR < 0 ? 0 : THR) : "memory");
        }
    }
}

int main() {
    const size_t bytes = (size_t)65536 * 21168;
    v4u* d;
    CHK(hipMalloc(&d, bytes + 65536));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) -> int {
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(a));
            for (int it = 0; it < 20; it++) launch();
            CHK(hipGetLastError());
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-34s %8.1f us/pass  %6.2f TB/s\n", name, ms * 1e3 / 20, bytes / (ms / 20 * 1e-3) / 1e12);
        }
        return 0;
    };
    char nm[64];
    for (int B : {21168, 42336}) {
        const int per16 = B / 16, nblk = (int)(bytes / B);
        for (int nw : {1, 2, 3, 4, 6, 8}) {
            snprintf(nm, sizeof nm, "blk %d nw %d K1 thr16", B, nw);
            run(nm, [&] { hipLaunchKernelGGL((k_pat<1, 16>), dim3(256), dim3(64 * nw), 0, 0, d, nblk, per16, nw); });
        }
        for (int nw : {2, 4, 6, 8}) {
            snprintf(nm, sizeof nm, "blk %d nw %d K2 thr16", B, nw);
            run(nm, [&] { hipLaunchKernelGGL((k_pat<2, 16>), dim3(256), dim3(64 * nw), 0, 0, d, nblk, per16, nw); });
        }
        for (int nw : {4, 8}) {
            snprintf(nm, sizeof nm, "blk %d nw %d K4 thr16", B, nw);
            run(nm, [&] { hipLaunchKernelGGL((k_pat<4, 16>), dim3(256), dim3(64 * nw), 0, 0, d, nblk, per16, nw); });
        }
        for (int nw : {2, 3, 4}) {
            snprintf(nm, sizeof nm, "blk %d nw %d K1 thr4", B, nw);
            run(nm, [&] { hipLaunchKernelGGL((k_pat<1, 4>), dim3(256), dim3(64 * nw), 0, 0, d, nblk, per16, nw); });
            snprintf(nm, sizeof nm, "blk %d nw %d K1 thr-1", B, nw);
            run(nm, [&] { hipLaunchKernelGGL((k_pat<1, -1>), dim3(256), dim3(64 * nw), 0, 0, d, nblk, per16, nw); });
        }
    }
    return 0;
}
