// Write-bandwidth ceiling probe (diagnostic, not part of the product): the fastest way this part
// writes the 1.39 GB C3 observation tensor, by store shape, grid and cache policy.
// hipcc --offload-arch=gfx950 -O3 -o storeceil tools/probe/storeceil.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// grid-stride 16 B per lane; U stores in flight per iteration; POL: 0 plain, 1 nontemporal
template <int U, int POL>
__global__ void __launch_bounds__(256) k_flat(v4u* o, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            v4u v = {(unsigned)i, 1u, 2u, 3u};
            if (POL) __builtin_nontemporal_store(v, o + i + u * stride);
            else o[i + u * stride] = v;
        }
    }
    for (; i < n16; i += stride) o[i] = v4u{0u, 0u, 0u, 0u};
}

// one wave writes a contiguous chunk of CH bytes, then the next chunk (wave-contiguous walk)
template <int CH, int POL>
__global__ void __launch_bounds__(256) k_chunk(v4u* o, size_t n16) {
    const int lane = threadIdx.x & 63;
    const size_t waves = (size_t)gridDim.x * 4, per = CH / 16;
    for (size_t c = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); c * per < n16; c += waves) {
        v4u* p = o + c * per;
#pragma unroll
        for (int k = lane; k < (int)per; k += 64) {
            v4u v = {(unsigned)k, 1u, 2u, 3u};
            if (c * per + k < n16) {
                if (POL) __builtin_nontemporal_store(v, p + k);
                else p[k] = v;
            }
        }
    }
}

// a workgroup (256 lanes) writes a contiguous chunk of CH bytes, 4 KB per workgroup instruction,
// then the next chunk gridDim.x chunks further (every workgroup's stream its own CH-byte block)
template <int CH>
__global__ void __launch_bounds__(256) k_wgchunk(v4u* o, size_t n16) {
    const size_t per = CH / 16;
    for (size_t c = blockIdx.x; c * per < n16; c += gridDim.x) {
        v4u* p = o + c * per;
        for (int k = threadIdx.x; k < (int)per; k += 256) {
            v4u v = {(unsigned)k, 1u, 2u, 3u};
            if (c * per + k < n16) p[k] = v;
        }
    }
}

// flat16 with at most T stores of this wave in flight (s_waitcnt vmcnt(T) after each store)
template <int T>
__global__ void __launch_bounds__(256) k_flat_thr(v4u* o, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        o[i] = v4u{(unsigned)i, 1u, 2u, 3u};
        if (T == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (T == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        if (T == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        if (T == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        if (T == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
}

// a workgroup of NT threads writes whole 21168-B env blocks cooperatively (16 B per thread per
// store), block b, b + gridDim.x, ...: the cooperative form of the observation flush
template <int NT>
__global__ void __launch_bounds__(NT) k_wgenv(v4u* o, int nblk) {
    constexpr int PER = 21168 / 16;
    for (int b = blockIdx.x; b < nblk; b += gridDim.x) {
        v4u* p = o + (size_t)b * PER;
#pragma unroll
        for (int i = 0; i < (PER + NT - 1) / NT; i++) {
            const int k = threadIdx.x + i * NT;
            if (k < PER) p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
        }
    }
}

// XCD-local patterns: workgroup b runs on XCD x = b % 8 (round-robin dispatch) and writes into the
// x-th eighth of the buffer.  MODE 0: flat 4-KB pieces among the XCD's workgroups; MODE 1: whole
// 21168-B env blocks per workgroup (cooperative), consecutive blocks for consecutive workgroups;
// MODE 2: whole env blocks per wave (the observation kernel's shape), consecutive waves consecutive blocks
template <int MODE>
__global__ void __launch_bounds__(256) k_xcd(v4u* o, int nblk) {
    constexpr int PER = 21168 / 16;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
    const int bx = nblk / 8;  // blocks per XCD
    v4u* base = o + (size_t)x * bx * PER;
    if (MODE == 0) {
        const size_t n = (size_t)bx * PER;
        for (size_t i = (size_t)j * 256 + threadIdx.x; i < n; i += (size_t)nj * 256) base[i] = v4u{(unsigned)i, 1u, 2u, 3u};
    } else if (MODE == 1) {
        for (int b = j; b < bx; b += nj) {
            v4u* p = base + (size_t)b * PER;
#pragma unroll
            for (int i = 0; i < (PER + 255) / 256; i++) {
                const int k = threadIdx.x + i * 256;
                if (k < PER) p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
            }
        }
    } else {
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        for (int b = j * 4 + w; b < bx; b += nj * 4) {
            v4u* p = base + (size_t)b * PER;
#pragma unroll
            for (int i = 0; i < (PER + 63) / 64; i++) {
                const int k = lane + i * 64;
                if (k < PER) p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
                if (MODE == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (MODE == 4) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                if (MODE == 5) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            }
        }
    }
}

int main() {
    const size_t bytes = (size_t)65536 * 21168;
    const size_t n16 = bytes / 16;
    v4u* d;
    CHK(hipMalloc(&d, bytes + 4096));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto run = [&](const char* name, int grid, auto launch) -> int {
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(a));
            for (int it = 0; it < 20; it++) launch(grid);
            CHK(hipGetLastError());
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-22s grid %6d %8.1f us/pass  %6.2f TB/s\n", name, grid, ms * 1e3 / 20, bytes / (ms / 20 * 1e-3) / 1e12);
        }
        return 0;
    };
    {
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(a));
            for (int it = 0; it < 20; it++) CHK(hipMemsetAsync(d, it, bytes, 0));
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-22s %8.1f us/pass  %6.2f TB/s\n", "hipMemsetAsync", ms * 1e3 / 20, bytes / (ms / 20 * 1e-3) / 1e12);
        }
    }
    for (int g : {128, 256, 384, 256 * 2, 256 * 4}) {
        run("flat16 u1", g, [&](int gr) { hipLaunchKernelGGL((k_flat<1, 0>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("flat16 u4", g, [&](int gr) { hipLaunchKernelGGL((k_flat<4, 0>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("flat16 u4 nt", g, [&](int gr) { hipLaunchKernelGGL((k_flat<4, 1>), dim3(gr), dim3(256), 0, 0, d, n16); });
    }
    for (int g : {256, 384, 256 * 2, 256 * 16}) {
        run("chunk 10584", g, [&](int gr) { hipLaunchKernelGGL((k_chunk<10576, 0>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("chunk 10584 nt", g, [&](int gr) { hipLaunchKernelGGL((k_chunk<10576, 1>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("chunk 4096", g, [&](int gr) { hipLaunchKernelGGL((k_chunk<4096, 0>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("chunk 21168", g, [&](int gr) { hipLaunchKernelGGL((k_chunk<21168, 0>), dim3(gr), dim3(256), 0, 0, d, n16); });
    }
    for (int g : {256, 512, 1024}) {
        run("xcd flat4k", g, [&](int gr) { hipLaunchKernelGGL((k_xcd<0>), dim3(gr), dim3(256), 0, 0, d, 65536); });
        run("xcd wgenv", g, [&](int gr) { hipLaunchKernelGGL((k_xcd<1>), dim3(gr), dim3(256), 0, 0, d, 65536); });
        run("xcd waveenv", g, [&](int gr) { hipLaunchKernelGGL((k_xcd<2>), dim3(gr), dim3(256), 0, 0, d, 65536); });
        run("xcd waveenv thr0", g, [&](int gr) { hipLaunchKernelGGL((k_xcd<3>), dim3(gr), dim3(256), 0, 0, d, 65536); });
        run("xcd waveenv thr1", g, [&](int gr) { hipLaunchKernelGGL((k_xcd<4>), dim3(gr), dim3(256), 0, 0, d, 65536); });
        run("xcd waveenv thr3", g, [&](int gr) { hipLaunchKernelGGL((k_xcd<5>), dim3(gr), dim3(256), 0, 0, d, 65536); });
    }
    for (int g : {128}) {
        run("wgenv 1024", g, [&](int gr) { hipLaunchKernelGGL((k_wgenv<1024>), dim3(gr), dim3(1024), 0, 0, d, 65536); });
        run("wgenv 512", g, [&](int gr) { hipLaunchKernelGGL((k_wgenv<512>), dim3(gr), dim3(512), 0, 0, d, 65536); });
        run("wgenv 256", g, [&](int gr) { hipLaunchKernelGGL((k_wgenv<256>), dim3(gr), dim3(256), 0, 0, d, 65536); });
    }
    for (int g : {2048}) {
        run("wgenv 256", g, [&](int gr) { hipLaunchKernelGGL((k_wgenv<256>), dim3(gr), dim3(256), 0, 0, d, 65536); });
        run("wgenv 512", g, [&](int gr) { hipLaunchKernelGGL((k_wgenv<512>), dim3(gr), dim3(512), 0, 0, d, 65536); });
    }
    for (int g : {256, 512}) {
        run("flat16 thr0", g, [&](int gr) { hipLaunchKernelGGL((k_flat_thr<0>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("flat16 thr1", g, [&](int gr) { hipLaunchKernelGGL((k_flat_thr<1>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("flat16 thr2", g, [&](int gr) { hipLaunchKernelGGL((k_flat_thr<2>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("flat16 thr4", g, [&](int gr) { hipLaunchKernelGGL((k_flat_thr<4>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("flat16 thr8", g, [&](int gr) { hipLaunchKernelGGL((k_flat_thr<8>), dim3(gr), dim3(256), 0, 0, d, n16); });
    }
    for (int g : {128, 1024}) {
        run("wgchunk 21168", g, [&](int gr) { hipLaunchKernelGGL((k_wgchunk<21168>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("wgchunk 42336", g, [&](int gr) { hipLaunchKernelGGL((k_wgchunk<42336>), dim3(gr), dim3(256), 0, 0, d, n16); });
        run("wgchunk 84672", g, [&](int gr) { hipLaunchKernelGGL((k_wgchunk<84672>), dim3(gr), dim3(256), 0, 0, d, n16); });
    }
    return 0;
}
