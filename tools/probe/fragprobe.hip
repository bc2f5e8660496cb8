// Probe (diagnostic, not the product): does the physical layout of a 1.39 GB output buffer change the C3
// observation stream's speed?  The writers' pattern of k_obs_ring (whole 21 168-B env blocks per wave, XCD-local,
// 3 writer waves per CU, 16-B stores) is timed into buffers allocated
//   fresh:  hipMalloc on an untouched device
//   frag:   hipMalloc after the device memory was cut up (many 1 MB buffers, every other one freed)
//   contig: hipExtMallocWithFlags(hipDeviceMallocContiguous) after the same fragmentation
//   hipcc --offload-arch=gfx950 -O3 -o fragprobe fragprobe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(192) k_writers(v4u* o, int nblk) {
    constexpr int PER = 21168 / 16, NW = 3;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
    const int bx = nblk / 8;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int b = j * NW + w; b < bx; b += nj * NW) {
        v4u* p = o + (size_t)(x * bx + b) * PER;
#pragma unroll 4
        for (int k = lane; k < PER; k += 64) {
            p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        }
    }
}

static int timeit(const char* name, v4u* d, int nblk) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e9f, tot = 0.f;
    for (int it = 0; it < 30; it++) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(k_writers, dim3(256), dim3(192), 0, 0, d, nblk);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (it >= 10) tot += ms;
        best = ms < best ? ms : best;
    }
    CHK(hipGetLastError());
    const double bytes = (double)nblk * 21168;
    printf("%-8s mean %7.1f us  best %7.1f us  %5.2f TB/s\n", name, tot * 1e3 / 20, best * 1e3, bytes / (tot / 20 * 1e-3) / 1e12);
    return 0;
}

int main() {
    const int nblk = 65536;
    const size_t bytes = (size_t)nblk * 21168;
    v4u* d = nullptr;
    CHK(hipMalloc(&d, bytes));
    if (timeit("fresh", d, nblk)) return 1;
    CHK(hipFree(d));
    // cut the free device memory up: 1 MB buffers over ~24 GB, every other one freed
    std::vector<void*> small;
    for (int i = 0; i < 24 * 1024; i++) {
        void* p = nullptr;
        if (hipMalloc(&p, 1 << 20) != hipSuccess) break;
        small.push_back(p);
    }
    for (size_t i = 0; i < small.size(); i += 2) CHK(hipFree(small[i]));
    printf("fragmented with %zu 1-MB buffers, half freed\n", small.size());
    CHK(hipMalloc(&d, bytes));
    if (timeit("frag", d, nblk)) return 1;
    CHK(hipFree(d));
    if (hipExtMallocWithFlags((void**)&d, bytes, hipDeviceMallocContiguous) == hipSuccess) {
        if (timeit("contig", d, nblk)) return 1;
        CHK(hipFree(d));
    } else {
        printf("contig: hipExtMallocWithFlags(hipDeviceMallocContiguous) failed\n");
    }
    for (size_t i = 1; i < small.size(); i += 2) CHK(hipFree(small[i]));
    CHK(hipMalloc(&d, bytes));
    if (timeit("again", d, nblk)) return 1;
    CHK(hipFree(d));
    return 0;
}
