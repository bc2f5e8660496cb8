// Write-pattern probe 3 (diagnostic, not part of the product): the C3 observation writers' shape
// (whole 21 168-B env blocks, 3 writer waves per workgroup, one workgroup per CU, XCD-local deal, 16
// stores in flight) with the flush's own pieces added one at a time: the chunk read from an LDS slot
// as int32 pairs and widened to int64 (LDS), raw buffer stores instead of global stores (BUF), and 12
// more waves per workgroup streaming reads at ~2 % of the written bytes (RD).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

template <bool LDS, bool BUF, bool RD>
__global__ void __launch_bounds__(960) k_w(v4u* o, int nblk, int per16, const unsigned* src, size_t nsrc) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
    const int bx = nblk / 8;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w >= 3) {  // readers
        if (!RD) return;
        unsigned acc = 0;
        const size_t per = nsrc / (gridDim.x * 12);
        const unsigned* s = src + (size_t)(blockIdx.x * 12 + (w - 3)) * per;
        for (size_t k = lane; k < per; k += 64) acc += s[k];
        if (acc == 0x12345678u) o[0] = v4u{acc, 0, 0, 0};
        return;
    }
    v4u* base = o + (size_t)x * bx * per16;
    const v2u* sv = (const v2u*)(smem + w * 16384);
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
    for (int b = j * 3 + w; b < bx; b += nj * 3) {
        const size_t off16 = (size_t)b * per16;
        for (int k = lane; k < per16; k += 64) {
            v4u v;
            if (LDS) {
                const v2u q = sv[k & 2047];
                v = v4u{q.x, (unsigned)((int)q.x >> 31), q.y, (unsigned)((int)q.y >> 31)};
            } else {
                v = v4u{(unsigned)k, 1u, 2u, 3u};
            }
            if (BUF) __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)((off16 + k) * 16 % 0x7fff0000u), 0, 0);
            else base[off16 + k] = v;
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        }
    }
}

int main() {
    const size_t bytes = (size_t)65536 * 21168;
    v4u* d;
    unsigned* src;
    const size_t nsrc = (size_t)26 << 20 >> 2;
    CHK(hipMalloc(&d, bytes + 65536));
    CHK(hipMalloc(&src, nsrc * 4));
    CHK(hipMemset(src, 1, nsrc * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const int per16 = 21168 / 16, nblk = 65536;
    auto run = [&](const char* name, auto kern, int threads) -> int {
        CHK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 3 * 16384));
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(a));
            for (int it = 0; it < 20; it++) hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 3 * 16384, 0, d, nblk, per16, src, nsrc);
            CHK(hipGetLastError());
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-28s %8.1f us/pass  %6.2f TB/s\n", name, ms * 1e3 / 20, bytes / (ms / 20 * 1e-3) / 1e12);
        }
        return 0;
    };
    run("global", k_w<false, false, false>, 192);
    run("global + LDS widen", k_w<true, false, false>, 192);
    run("buffer", k_w<false, true, false>, 192);
    run("buffer + LDS widen", k_w<true, true, false>, 192);
    run("global + readers", k_w<false, false, true>, 960);
    run("buffer + LDS widen + readers", k_w<true, true, true>, 960);
    run("global (15 waves, 12 idle)", k_w<false, false, false>, 960);
    return 0;
}
