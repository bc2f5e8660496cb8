// Write-policy probe (diagnostic, not part of the product): the C3 observation writers' pattern (whole
// 21 168-B env blocks per wave, XCD-local, 3 writer waves per CU, 16 stores in flight) with the global
// store's cache-policy bits varied, alone and with "readers": per env block, the writer wave first reads
// 384 B of a 26 MB state array the previous kernel wrote (the encoders' per-env state loads in k_obs_ring,
// 65 536 envs x ~400 B).  Does a store policy that keeps the 1.39 GB stream out of the caches let those
// reads hit in cache, and what does each policy cost the stream itself?
//   hipcc --offload-arch=gfx950 -O3 -o storepol storepol.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st16(v4u* p, v4u v) {
    if constexpr (POL == 0) {
        *p = v;
    } else if constexpr (POL == 1) {
        asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (POL == 2) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (POL == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (POL == 4) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    } else {
        asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
    }
}

// state[e] = 96 words per env (384 B), written by k_state, read per env block by the writers (READ)
__global__ void k_state(unsigned* st, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        st[i] = (unsigned)i * 2654435761u;
}

template <int POL, bool READ>
__global__ void __launch_bounds__(192) k_writers(v4u* o, const unsigned* st, int nblk, unsigned* sink) {
    constexpr int PER = 21168 / 16, NW = 3;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
    const int bx = nblk / 8;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (int b = j * NW + w; b < bx; b += nj * NW) {
        const int e = x * bx + b;
        v4u* p = o + (size_t)e * PER;
        unsigned s0 = 0;
        if (READ) {  // 384 B of the env's state: 1.5 words per lane, like the encoders' row loads
            s0 = st[(size_t)e * 96 + lane];
            if (lane < 32) s0 += st[(size_t)e * 96 + 64 + lane];
        }
#pragma unroll 4
        for (int k = lane; k < PER; k += 64) {
            st16<POL>(p + k, v4u{(unsigned)k + s0, 1u, 2u, 3u});
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        }
        acc += s0;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const int nblk = 65536;
    const size_t bytes = (size_t)nblk * 21168, sw = (size_t)nblk * 96;
    v4u* d;
    unsigned *st, *sink;
    CHK(hipMalloc(&d, bytes + 65536));
    CHK(hipMalloc(&st, sw * 4));
    CHK(hipMalloc(&sink, 64));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) -> int {
        float tot = 0;
        for (int rep = 0; rep < 2; rep++) {
            tot = 0;
            for (int it = 0; it < 20; it++) {
                hipLaunchKernelGGL(k_state, dim3(1024), dim3(256), 0, 0, st, sw);  // the tick's state writes
                CHK(hipEventRecord(a));
                launch();
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                float ms;
                CHK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
            }
            CHK(hipGetLastError());
        }
        printf("%-28s %8.1f us/pass  %6.2f TB/s\n", name, tot * 1e3 / 20, bytes / (tot / 20 * 1e-3) / 1e12);
        return 0;
    };
#define RUN(P, R, name) run(name, [&] { hipLaunchKernelGGL((k_writers<P, R>), dim3(256), dim3(192), 0, 0, d, st, nblk, sink); })
    RUN(0, false, "default");
    RUN(0, true, "default + reads");
    RUN(1, false, "nt");
    RUN(1, true, "nt + reads");
    RUN(2, false, "sc1");
    RUN(2, true, "sc1 + reads");
    RUN(3, false, "sc0 sc1");
    RUN(3, true, "sc0 sc1 + reads");
    RUN(4, false, "sc1 nt");
    RUN(4, true, "sc1 nt + reads");
    RUN(5, false, "sc0");
    RUN(5, true, "sc0 + reads");
    return 0;
}
