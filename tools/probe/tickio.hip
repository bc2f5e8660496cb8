// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for k_tick's access pattern (diagnostic only).
// MI355X_MICROARCH.md: FETCH_SIZE reads half the bytes of 16-B-per-lane streaming loads; other widths
// are uncalibrated.  k_tick moves narrow SoA elements (4 B and 1 B per lane, 8 consecutive envs of one
// slot per one-wave workgroup at G = 8), so its counters are compared here with a kernel that moves
// exactly the tick's state rows, with the tick's lane mapping and none of its work: the bytes it moves
// are known, so counter / bytes is the factor to apply to k_tick's counters.
//   hipcc --offload-arch=gfx950 -O3 -o tickio tools/probe/tickio.hip
//   rocprofv3 --pmc FETCH_SIZE -- ./tickio ; rocprofv3 --pmc WRITE_SIZE -- ./tickio
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                                \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));           \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

constexpr int N = 65536, E = 12, A = 2, G = 8, NE = 64 / G, OW = 14, RW = 32, NSC = 9;

struct Rows {
    int32_t *pos, *life, *scal, *prev, *act, *opres;
    uint8_t *weap, *pres, *ord, *listed;
    uint32_t* ring;  // [N][1248]
    uint32_t* rngst;
    int32_t* sink;
};

// tick_io: the stage-in reads and stage-out writes of k_tick<8> at C3 (entity SoA, scalar rows,
// tracker rows, actions, obstacle-present bits, a 32-word window of the env's MT ring at its offset)
// the engine's XCD-contiguous workgroup order (zs_obs.hpp xcd_remap): each XCD's L2 sees a contiguous
// range of envs, as in k_tick
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

__global__ void __launch_bounds__(64) k_tick_io(Rows r, int write) {
    const int lane = threadIdx.x, g = lane / G, j = lane % G, e = xcd_remap(blockIdx.x, gridDim.x) * NE + g;
    int32_t acc = 0;
    for (int s = j; s < E; s += G) {
        acc += r.pos[(size_t)s * N + e] + r.life[(size_t)s * N + e] + r.weap[(size_t)s * N + e] +
               r.pres[(size_t)s * N + e] + r.ord[(size_t)s * N + e];
    }
    for (int f = j; f < NSC; f += G) acc += r.scal[(size_t)f * N + e];
    for (int a = j; a < A; a += G) acc += r.prev[(size_t)a * N + e] + r.listed[(size_t)a * N + e];
    for (int k = j; k < 3 * A; k += G) acc += r.act[(size_t)e * 3 * A + k];
    for (int w = j; w < OW; w += G) acc += r.opres[(size_t)e * OW + w];
    const uint32_t st = r.rngst[e], off = st % 500;
    for (int k = j; k < RW; k += G) acc += (int32_t)r.ring[(size_t)e * 1248 + off + k];
    if (!write) {
        if (acc == 0x7fffffff) r.sink[0] = acc;
        return;
    }
    for (int s = j; s < E; s += G) {
        r.pos[(size_t)s * N + e] = acc;
        r.life[(size_t)s * N + e] = acc + 1;
        r.weap[(size_t)s * N + e] = (uint8_t)acc;
        r.pres[(size_t)s * N + e] = (uint8_t)(acc >> 8);
        r.ord[(size_t)s * N + e] = (uint8_t)(acc >> 16);
    }
    for (int f = j; f < NSC; f += G) r.scal[(size_t)f * N + e] = acc;
    for (int a = j; a < A; a += G) {
        r.prev[(size_t)a * N + e] = acc;
        r.listed[(size_t)a * N + e] = 1;
    }
    if (j == 0) r.rngst[e] = st + 12;
}

int main() {
    Rows r;
    CHK(hipMalloc(&r.pos, 4ull * E * N));
    CHK(hipMalloc(&r.life, 4ull * E * N));
    CHK(hipMalloc(&r.scal, 4ull * NSC * N));
    CHK(hipMalloc(&r.prev, 4ull * A * N));
    CHK(hipMalloc(&r.act, 4ull * 3 * A * N));
    CHK(hipMalloc(&r.opres, 4ull * OW * N));
    CHK(hipMalloc(&r.weap, 1ull * E * N));
    CHK(hipMalloc(&r.pres, 1ull * E * N));
    CHK(hipMalloc(&r.ord, 1ull * E * N));
    CHK(hipMalloc(&r.listed, 1ull * A * N));
    CHK(hipMalloc(&r.ring, 4ull * 1248 * N));
    CHK(hipMalloc(&r.rngst, 4ull * N));
    CHK(hipMalloc(&r.sink, 4));
    CHK(hipMemset(r.rngst, 0, 4ull * N));
    // a 1 GB buffer written between launches: every launch starts with cold caches (L2 and the 256 MB
    // Infinity Cache), as k_tick does behind the 1.39 GB observation stream
    uint8_t* flush;
    const size_t FB = 1ull << 30;
    CHK(hipMalloc(&flush, FB));
    const double rd = (double)N * (E * 11 + NSC * 4 + A * 5 + 3 * A * 4 + OW * 4 + RW * 4 + 4);
    const double wr = (double)N * (E * 11 + NSC * 4 + A * 5) + (double)N / G * 4;  // rngst by one lane per env
    for (int rep = 0; rep < 5; rep++) {
        CHK(hipMemsetAsync(flush, rep, FB, 0));
        hipLaunchKernelGGL(k_tick_io, dim3(N / NE), dim3(64), 0, 0, r, 0);
        CHK(hipMemsetAsync(flush, rep + 7, FB, 0));
        hipLaunchKernelGGL(k_tick_io, dim3(N / NE), dim3(64), 0, 0, r, 1);
    }
    CHK(hipDeviceSynchronize());
    printf("k_tick_io read-only launch: %.0f bytes read; read+write launch: %.0f read, %.0f written (rngst "
           "by one lane of %d)\n", rd, rd, (double)N * (E * 11 + NSC * 4 + A * 5) + 4.0 * N, G);
    (void)wr;
    return 0;
}
