// Write-pattern probe for the observation store stream (diagnostic, not part of the product): the C3
// observation tensor (65 536 env blocks of 21 168 B) written by one workgroup per CU with the writer
// topologies an encoder/writer kernel can realise.  Every env block is written by one CU (its encoder
// holds the env in LDS); what varies is how the CU's writer waves split the block and how envs are
// dealt to CUs.
//   hipcc --offload-arch=gfx950 -O3 -o envstore tools/probe/envstore.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int PER = 21168 / 16;  // 16-B chunks per env block

// env of round k for workgroup b: DEAL 0 = chip-strided (b', b' + G, ... with b' XCD-contiguous);
// DEAL 1 = XCD regions, W consecutive envs per workgroup per round
template <int DEAL>
__device__ __forceinline__ int env_of(int b, int nb, int n, int W, int u, int& cnt) {
    const int q = nb >> 3, r = nb & 7, x = b & 7, j = b >> 3;
    const int gs = x * q + (x < r ? x : r), gx = q + (x < r);
    if (DEAL == 0) {
        const int g = gs + j;
        const int units = (n + W - 1) / W;  // W consecutive envs per unit
        const int uc = g < units ? (units - g + nb - 1) / nb : 0;
        cnt = uc * W;
        return (g + (u / W) * nb) * W + u % W;
    }
    const int r0 = (int)((long long)n * gs / nb), r1 = (int)((long long)n * (gs + gx) / nb);
    const int span = gx * W, off = j * W, m = r1 - r0 - off;
    cnt = m <= 0 ? 0 : (m / span) * W + min(m % span, W);
    return r0 + (u / W) * span + off + u % W;
}

// A: NW writer waves, each streams whole env blocks of its own (wave w: the CU's envs w, w + NW, ...)
template <int NW, int DEAL>
__global__ void __launch_bounds__(64 * NW) k_own(v4u* o, int n) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int cnt;
    env_of<DEAL>(blockIdx.x, gridDim.x, n, NW, 0, cnt);
    for (int u = w; u < cnt; u += NW) {
        int c2;
        v4u* p = o + (size_t)env_of<DEAL>(blockIdx.x, gridDim.x, n, NW, u, c2) * PER;
#pragma unroll
        for (int i = 0; i < (PER + 63) / 64; i++) {
            const int k = lane + 64 * i;
            if (k < PER) p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
        }
    }
}

// B: the NW waves write one env block together, 1-KB pieces dealt round-robin (wave w: pieces w, w + NW, ...)
// C: the NW waves write one env block together, wave w a contiguous 1/NW of it
template <int NW, int MODE>
__global__ void __launch_bounds__(64 * NW) k_coop(v4u* o, int n) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int cnt;
    env_of<1>(blockIdx.x, gridDim.x, n, 1, 0, cnt);
    constexpr int NP = (PER + 63) / 64, QP = (NP + NW - 1) / NW;
    for (int u = 0; u < cnt; u++) {
        int c2;
        v4u* p = o + (size_t)env_of<1>(blockIdx.x, gridDim.x, n, 1, u, c2) * PER;
#pragma unroll
        for (int i = 0; i < QP; i++) {
            const int piece = MODE == 0 ? w + NW * i : w * QP + i;
            const int k = lane + 64 * piece;
            if (piece < NP && k < PER) p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
        }
    }
}

// D: a workgroup's envs in pairs: NW waves over 2 adjacent env blocks as one contiguous 42-KB stream
// (wave w pieces w, w + NW, ...), the XCD's workgroups on consecutive pairs
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_pair(v4u* o, int n) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int cnt;
    env_of<1>(blockIdx.x, gridDim.x, n / 2, 1, 0, cnt);
    constexpr int NP = (2 * PER + 63) / 64, QP = (NP + NW - 1) / NW;
    for (int u = 0; u < cnt; u++) {
        int c2;
        v4u* p = o + (size_t)env_of<1>(blockIdx.x, gridDim.x, n / 2, 1, u, c2) * 2 * PER;
#pragma unroll
        for (int i = 0; i < QP; i++) {
            const int piece = w + NW * i;
            const int k = lane + 64 * piece;
            if (piece < NP && k < 2 * PER) p[k] = v4u{(unsigned)k, 1u, 2u, 3u};
        }
    }
}

int main(int argc, char** argv) {
    const int n = 65536;
    const size_t bytes = (size_t)n * 21168;
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto run = [&](const char* name, v4u* d, int grid, auto launch) -> int {
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(a));
            for (int it = 0; it < 20; it++) launch(d, grid);
            CHK(hipGetLastError());
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-26s %p grid %5d %8.1f us/pass  %6.2f TB/s\n", name, (void*)d, grid, ms * 1e3 / 20, bytes / (ms / 20 * 1e-3) / 1e12);
        }
        return 0;
    };
    if (argc > 1) {
        // placement: the same pattern into several separately allocated buffers
        // argv[2]: 0 hipMalloc, 1 hipExtMallocWithFlags(hipDeviceMallocContiguous), 2 VMM (hipMemCreate of
        // the whole size, mapped at a reserved range), 3 hipMalloc of 4 GiB
        const int nb = atoi(argv[1]), mode = argc > 2 ? atoi(argv[2]) : 0;
        v4u* bufs[16];
        for (int i = 0; i < nb && i < 16; i++) {
            if (mode == 1) {
                CHK(hipExtMallocWithFlags((void**)&bufs[i], bytes + 4096, hipDeviceMallocContiguous));
            } else if (mode == 2) {
                hipMemAllocationProp prop = {};
                prop.type = hipMemAllocationTypePinned;
                prop.location.type = hipMemLocationTypeDevice;
                prop.location.id = 0;
                size_t gran = 0;
                CHK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
                const size_t sz = (bytes + 4096 + gran - 1) / gran * gran;
                if (i == 0) printf("VMM granularity %zu\n", gran);
                hipMemGenericAllocationHandle_t hdl;
                void* va = nullptr;
                CHK(hipMemAddressReserve(&va, sz, 0, nullptr, 0));
                CHK(hipMemCreate(&hdl, sz, &prop, 0));
                CHK(hipMemMap(va, sz, 0, hdl, 0));
                hipMemAccessDesc acc = {};
                acc.location = prop.location;
                acc.flags = hipMemAccessFlagsProtReadWrite;
                CHK(hipMemSetAccess(va, sz, &acc, 1));
                bufs[i] = (v4u*)va;
            } else if (mode == 3) {
                CHK(hipMalloc(&bufs[i], 4ull << 30));
            } else {
                CHK(hipMalloc(&bufs[i], bytes + 4096));
            }
            CHK(hipMemset(bufs[i], 0, bytes));
        }
        for (int i = 0; i < nb && i < 16; i++) {
            run("own 4 waves xcd", bufs[i], 256, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_own<4, 1>), dim3(gr), dim3(256), 0, 0, d, n); });
            run("flat4k-like coop quarters", bufs[i], 256, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_coop<4, 1>), dim3(gr), dim3(256), 0, 0, d, n); });
        }
        return 0;
    }
    v4u* d;
    CHK(hipMalloc(&d, bytes + 4096));
    for (int g : {256, 512}) {
        run("own 1 wave  chip", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_own<1, 0>), dim3(gr), dim3(64), 0, 0, d, n); });
        run("own 1 wave  xcd", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_own<1, 1>), dim3(gr), dim3(64), 0, 0, d, n); });
        run("own 2 waves xcd", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_own<2, 1>), dim3(gr), dim3(128), 0, 0, d, n); });
        run("own 4 waves chip", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_own<4, 0>), dim3(gr), dim3(256), 0, 0, d, n); });
        run("own 4 waves xcd", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_own<4, 1>), dim3(gr), dim3(256), 0, 0, d, n); });
        run("own 8 waves xcd", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_own<8, 1>), dim3(gr), dim3(512), 0, 0, d, n); });
        run("coop 4 rr1k", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_coop<4, 0>), dim3(gr), dim3(256), 0, 0, d, n); });
        run("coop 4 quarters", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_coop<4, 1>), dim3(gr), dim3(256), 0, 0, d, n); });
        run("pair 4 rr1k", d, g, [&](v4u* d, int gr) { hipLaunchKernelGGL((k_pair<4>), dim3(gr), dim3(256), 0, 0, d, n); });
    }
    return 0;
}
