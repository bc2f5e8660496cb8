// Store-bandwidth probe for the observation write shape (diagnostic, not part of the product).
// 65536 envs x [2 agents][3 channels][441 cells] int64 = 1.39 GB per pass, written as
//   k_cells8 : one wave per env, lane = cell, 3 x 8 B stores per cell (k_obs's shape)
//   k_pairs16: one wave per env, lane = 2 adjacent values, 16 B stores over the env's flat block
//   k_flat16 : grid-stride 16 B per lane over the whole buffer (memset shape)
// hipcc --offload-arch=gfx950 -O3 -o storebw tools/probe/storebw.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NE = 65536, NA = 2, PL = 441, PER = NA * 3 * PL;  // int64 values per env

__global__ void __launch_bounds__(256) k_cells8(int64_t* out, int n) {
    int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= n) return;
    for (int a = 0; a < NA; a++) {
        int64_t* o = out + ((size_t)e * NA + a) * 3 * PL;
        for (int c = lane; c < PL; c += 64) {
            o[c] = c;
            o[PL + c] = e;
            o[2 * PL + c] = a;
        }
    }
}

__device__ __forceinline__ int xremap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

// k_cells8 with XCD-contiguous env ranges
__global__ void __launch_bounds__(256) k_cells8x(int64_t* out, int n) {
    int e = xremap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= n) return;
    for (int a = 0; a < NA; a++) {
        int64_t* o = out + ((size_t)e * NA + a) * 3 * PL;
        for (int c = lane; c < PL; c += 64) {
            o[c] = c;
            o[PL + c] = e;
            o[2 * PL + c] = a;
        }
    }
}

// k_cells8 after staging RB bytes of per-env state into LDS (the encoder's read side)
constexpr int RB = 2304;
__global__ void __launch_bounds__(256) k_cells8r(int64_t* out, const int* st, int n) {
    __shared__ int img[4][RB / 4];
    int w = threadIdx.x >> 6, e = blockIdx.x * 4 + w, lane = threadIdx.x & 63;
    if (e >= n) return;
    const int* src = st + (size_t)e * (RB / 4);
    int v[RB / 4 / 64];
#pragma unroll
    for (int i = 0; i < RB / 4 / 64; i++) v[i] = src[lane + 64 * i];
#pragma unroll
    for (int i = 0; i < RB / 4 / 64; i++) img[w][lane + 64 * i] = v[i];
    __builtin_amdgcn_wave_barrier();
    for (int a = 0; a < NA; a++) {
        int64_t* o = out + ((size_t)e * NA + a) * 3 * PL;
        for (int c = lane; c < PL; c += 64) {
            int x = img[w][(c * 7) % (RB / 4)];
            o[c] = x;
            o[PL + c] = e;
            o[2 * PL + c] = a;
        }
    }
}

__global__ void __launch_bounds__(256) k_pairs16(int64_t* out, int n) {
    int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= n) return;
    longlong2* o = (longlong2*)(out + (size_t)e * PER);
    for (int i = lane; i < PER / 2; i += 64) o[i] = make_longlong2(i, e);
}

__global__ void __launch_bounds__(256) k_flat16(int64_t* out, size_t n2) {
    longlong2* o = (longlong2*)out;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256)
        o[i] = make_longlong2(i, 1);
}

int main() {
    size_t bytes = (size_t)NE * PER * 8;
    int64_t* d;
    CHK(hipMalloc(&d, bytes));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    int* st;
    CHK(hipMalloc(&st, (size_t)NE * RB));
    CHK(hipMemset(st, 1, (size_t)NE * RB));
    const char* names[5] = {"cells8", "pairs16", "flat16", "cells8x", "cells8r"};
    for (int k = 0; k < 5; k++) {
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(a));
            for (int it = 0; it < 20; it++) {
                if (k == 0) hipLaunchKernelGGL(k_cells8, dim3(NE / 4), dim3(256), 0, 0, d, NE);
                else if (k == 1) hipLaunchKernelGGL(k_pairs16, dim3(NE / 4), dim3(256), 0, 0, d, NE);
                else if (k == 2) hipLaunchKernelGGL(k_flat16, dim3(256 * 32), dim3(256), 0, 0, d, bytes / 16);
                else if (k == 3) hipLaunchKernelGGL(k_cells8x, dim3(NE / 4), dim3(256), 0, 0, d, NE);
                else hipLaunchKernelGGL(k_cells8r, dim3(NE / 4), dim3(256), 0, 0, d, st, NE);
            }
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-10s %8.1f us/pass  %6.2f TB/s (written)\n", names[k], ms * 1e3 / 20,
                            bytes / (ms / 20 * 1e-3) / 1e12);
        }
    }
    return 0;
}
