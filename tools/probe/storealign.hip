// Write-pattern probe 3 (diagnostic, not part of the product): does the 16-B store stream of one block per
// wave lose bandwidth to blocks that start off a 128-B line?  The observation writers stream 21 168-B env
// blocks (21 168 mod 128 = 48: every block but one in eight starts and ends inside a line another wave
// writes).  XCD-local walk as the ring's deal (workgroup b on XCD b % 8 writes the x-th eighth of the
// buffer, consecutive waves of an XCD on consecutive blocks), NW writer waves per workgroup, one
// workgroup per CU.  Modes:
//   B-byte blocks per wave (B = 21168 misaligned, 21248 = 166 lines, 20480 = 5 x 4 KB);
//   "grp": NW consecutive 21 168-B blocks of a workgroup re-cut into NW contiguous ranges at 256-B
//   boundaries (each wave streams one aligned range; only the group's two ends stay unaligned).
//   hipcc --offload-arch=gfx950 -O3 -o storealign storealign.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int THR>
__device__ __forceinline__ void thr() {
    if (THR >= 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(THR < 0 ? 0 : THR) : "memory");
}

// whole B-byte blocks per wave; writes elements [k0, k1) of 16 B within the region
template <int THR>
__global__ void __launch_bounds__(1024) k_blocks(v4u* o, size_t total16, int per16, int nw) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
    const size_t nblk = total16 / per16, bx = nblk / 8;
    v4u* base = o + (size_t)x * bx * per16;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w >= nw) return;
    for (size_t b = (size_t)j * nw + w; b < bx; b += (size_t)nj * nw) {
        v4u* p = base + b * per16;
        for (int k = lane; k < per16; k += 64) {
            p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
            thr<THR>();
        }
    }
}

// a workgroup's NW consecutive 21 168-B blocks (one group) cut into NW ranges at 256-B boundaries;
// byte-exact ends via 16-B stores (21 168 is a multiple of 16)
template <int THR>
__global__ void __launch_bounds__(1024) k_group(v4u* o, size_t total16, int per16, int nw) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
    const size_t nblk = total16 / per16, bx = nblk / 8;
    v4u* base = o + (size_t)x * bx * per16;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w >= nw) return;
    const size_t ngrp = bx / nw;
    for (size_t g = j; g < ngrp; g += nj) {
        const size_t s16 = g * nw * per16, e16 = s16 + (size_t)nw * per16;  // group range in 16-B units
        const uintptr_t sb = (uintptr_t)(base + s16), eb = (uintptr_t)(base + e16);
        // cut points: w / nw of the way, rounded down to 256 B (absolute addresses)
        auto cut = [&](int i) -> size_t {
            if (i == 0) return s16;
            if (i == nw) return e16;
            uintptr_t a = sb + (eb - sb) * i / nw;
            a &= ~(uintptr_t)255;
            return (size_t)((v4u*)a - base);
        };
        const size_t k0 = cut(w), k1 = cut(w + 1);
        for (size_t k = k0 + lane; k < k1; k += 64) {
            base[k] = v4u{(unsigned)k, 1u, 2u, 3u};
            thr<THR>();
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
            if (rep) printf("%-40s %8.1f us/pass  %6.2f TB/s\n", name, ms * 1e3 / 20, bytes / (ms / 20 * 1e-3) / 1e12);
        }
        return 0;
    };
    char nm[96];
    const size_t total16 = bytes / 16;
    for (int nw : {2, 3, 4}) {
        for (int B : {21168, 21248, 20480, 21504}) {
            snprintf(nm, sizeof nm, "blocks %d B nw %d thr16", B, nw);
            run(nm, [&] { hipLaunchKernelGGL((k_blocks<16>), dim3(256), dim3(64 * nw), 0, 0, d, total16, B / 16, nw); });
        }
        snprintf(nm, sizeof nm, "group of %d x 21168 B, 256-B cuts thr16", nw);
        run(nm, [&] { hipLaunchKernelGGL((k_group<16>), dim3(256), dim3(64 * nw), 0, 0, d, total16, 21168 / 16, nw); });
        snprintf(nm, sizeof nm, "group of %d x 21168 B, 256-B cuts thr4", nw);
        run(nm, [&] { hipLaunchKernelGGL((k_group<4>), dim3(256), dim3(64 * nw), 0, 0, d, total16, 21168 / 16, nw); });
    }
    // the same with the buffer itself offset by 48 B (the first block starts off a line, like an unaligned env)
    for (int nw : {3}) {
        snprintf(nm, sizeof nm, "blocks 21248 B nw %d, base +48 B", nw);
        run(nm, [&] { hipLaunchKernelGGL((k_blocks<16>), dim3(256), dim3(64 * nw), 0, 0, (v4u*)((char*)d + 48), total16 - 4, 21248 / 16, nw); });
    }
    return 0;
}
