// Store-bandwidth probe for the observation write shape (diagnostic, not part of the product).
// 65536 envs x [2 agents][3 channels][441 cells] int64 = 1.39 GB per pass, written as
//   cells8   : one wave per env, lane = cell, 3 x 8 B stores per cell (k_obs's shape)
//   cells8nt : the same with nontemporal stores
//   pairs16  : one wave per env, lane = 2 adjacent values, 16 B stores over the env's flat block
//   pairs16nt: the same, nontemporal
//   lds16    : one wave per env, values written to an LDS copy of the env block (8 B per cell and
//              channel, k_obs's compute shape), then streamed out 16 B per lane
//   flat16   : grid-stride 16 B per lane over the whole buffer (memset shape)
//   p_*      : persistent grids (256 x K workgroups walking envs) of the same bodies
// hipcc --offload-arch=gfx950 -O3 -o storebw tools/probe/storebw.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NE = 65536, NA = 2, PL = 441, PER = NA * 3 * PL;  // int64 values per env

template <bool NT>
__device__ __forceinline__ void st8(int64_t* p, int64_t v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NT>
__device__ __forceinline__ void body_cells8(int64_t* out, int e, int lane) {
    for (int a = 0; a < NA; a++) {
        int64_t* o = out + ((size_t)e * NA + a) * 3 * PL;
        for (int c = lane; c < PL; c += 64) {
            st8<NT>(o + c, c);
            st8<NT>(o + PL + c, e);
            st8<NT>(o + 2 * PL + c, a);
        }
    }
}

template <bool NT>
__device__ __forceinline__ void body_pairs16(int64_t* out, int e, int lane) {
    // env block starts 8-B aligned only for odd e (PER is even: 2646 values = 21168 B, 16-B aligned)
    typedef long long v2i64 __attribute__((ext_vector_type(2)));
    v2i64* o = (v2i64*)(out + (size_t)e * PER);
    for (int i = lane; i < PER / 2; i += 64) {
        v2i64 v = {(long long)i, (long long)e};
        if (NT) __builtin_nontemporal_store(v, o + i);
        else o[i] = v;
    }
}

__device__ __forceinline__ void body_lds16(int64_t* out, int e, int lane, int64_t* img) {
    for (int a = 0; a < NA; a++) {
        for (int c = lane; c < PL; c += 64) {
            img[a * 3 * PL + c] = c;
            img[a * 3 * PL + PL + c] = e;
            img[a * 3 * PL + 2 * PL + c] = a;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const longlong2* s = (const longlong2*)img;
    longlong2* o = (longlong2*)(out + (size_t)e * PER);
    for (int i = lane; i < PER / 2; i += 64) o[i] = s[i];
    __builtin_amdgcn_wave_barrier();
}

template <int K>
__global__ void __launch_bounds__(256) k_one(int64_t* out, int n) {
    __shared__ int64_t img[K == 4 ? 4 : 1][K == 4 ? PER : 1];
    int w = threadIdx.x >> 6, e = blockIdx.x * 4 + w, lane = threadIdx.x & 63;
    if (e >= n) return;
    if (K == 0) body_cells8<false>(out, e, lane);
    if (K == 1) body_cells8<true>(out, e, lane);
    if (K == 2) body_pairs16<false>(out, e, lane);
    if (K == 3) body_pairs16<true>(out, e, lane);
    if (K == 4) body_lds16(out, e, lane, img[w]);
}

template <int K>
__global__ void __launch_bounds__(256) k_pers(int64_t* out, int n) {
    __shared__ int64_t img[K == 4 ? 4 : 1][K == 4 ? PER : 1];
    int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int e = blockIdx.x * 4 + w; e < n; e += gridDim.x * 4) {
        if (K == 0) body_cells8<false>(out, e, lane);
        if (K == 1) body_cells8<true>(out, e, lane);
        if (K == 2) body_pairs16<false>(out, e, lane);
        if (K == 3) body_pairs16<true>(out, e, lane);
        if (K == 4) body_lds16(out, e, lane, img[w]);
    }
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
    struct V { const char* name; int kind; int grid; };
    V vs[] = {{"cells8", 0, NE / 4},  {"cells8nt", 1, NE / 4},  {"pairs16", 2, NE / 4}, {"pairs16nt", 3, NE / 4},
              {"lds16", 4, NE / 4},   {"p_cells8", 10, 256 * 8}, {"p_cells8nt", 11, 256 * 8},
              {"p_pairs16", 12, 256 * 8}, {"p_pairs16nt", 13, 256 * 8}, {"p_lds16", 14, 256 * 2},
              {"p_pairs16_g4", 12, 256 * 4}, {"p_pairs16_g16", 12, 256 * 16}, {"flat16", 20, 256 * 32}};
    for (const V& v : vs) {
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(a));
            for (int it = 0; it < 20; it++) {
                switch (v.kind) {
                case 0: hipLaunchKernelGGL(k_one<0>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 1: hipLaunchKernelGGL(k_one<1>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 2: hipLaunchKernelGGL(k_one<2>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 3: hipLaunchKernelGGL(k_one<3>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 4: hipLaunchKernelGGL(k_one<4>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 10: hipLaunchKernelGGL(k_pers<0>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 11: hipLaunchKernelGGL(k_pers<1>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 12: hipLaunchKernelGGL(k_pers<2>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 13: hipLaunchKernelGGL(k_pers<3>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                case 14: hipLaunchKernelGGL(k_pers<4>, dim3(v.grid), dim3(256), 0, 0, d, NE); break;
                default: hipLaunchKernelGGL(k_flat16, dim3(v.grid), dim3(256), 0, 0, d, bytes / 16); break;
                }
            }
            CHK(hipGetLastError());
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-14s grid %6d %8.1f us/pass  %6.2f TB/s (written)\n", v.name, v.grid, ms * 1e3 / 20,
                            bytes / (ms / 20 * 1e-3) / 1e12);
        }
    }
    return 0;
}
