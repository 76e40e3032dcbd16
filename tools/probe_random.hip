// probe_random.hip — rates of random 4-B accesses on MI355X, to size the
// delivery path's seen-set design.
//
// Every lane touches one pseudo-random u32 cell of a table of `bytes`; a
// wave-instruction therefore hits 64 different lines (the delivery claim
// pattern).  Modes:
//   load      plain load, summed
//   store     plain store
//   amin_nr   atomicMin, no return
//   amin_r    atomicMin, result used
//   cas64     64-bit CAS loop (x -> x + 1), result used
//   cas64_row 64-bit CAS loop, 8 lanes of each 32-lane group hitting one
//             256-B row (the transposed counter pattern)
// build: hipcc --offload-arch=gfx950 -O3 tools/probe_random.hip -o tools/probe_random
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(uint32_t* tab, uint64_t ncell, uint64_t nops, uint32_t* sink, uint32_t salt)
{
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nops; i += stride) {
        uint64_t c;
        if (MODE == 5) {
            // groups of 32 lanes: 8 active lanes in one 256-B row
            const uint64_t grp = i >> 5;
            const uint32_t l = (uint32_t)(i & 31);
            if ((l & 3) != 0) continue;
            c = ((uint64_t)mix(grp * 0x9E3779B97F4A7C15ull + salt) % (ncell / 64)) * 64 + l * 2;
        } else {
            c = (uint64_t)mix(i * 0x9E3779B97F4A7C15ull + salt) % ncell;
        }
        if (MODE == 0) acc += tab[c];
        if (MODE == 1) tab[c] = (uint32_t)i;
        if (MODE == 2) atomicMin(&tab[c], (uint32_t)i);
        if (MODE == 3) acc += atomicMin(&tab[c], (uint32_t)i);
        if (MODE == 4 || MODE == 5) {
            unsigned long long* q = reinterpret_cast<unsigned long long*>(tab) + (c >> 1);
            unsigned long long old = *q;
            for (;;) {
                const unsigned long long prev = atomicCAS(q, old, old + 1);
                if (prev == old) break;
                old = prev;
            }
            acc += (uint32_t)old;
        }
    }
    if (acc == 0xdeadbeef) sink[0] = acc;
}

template <int MODE>
static float run(uint32_t* tab, uint64_t ncell, uint64_t nops, uint32_t* sink, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_probe<MODE>, dim3(2048), dim3(256), 0, 0, tab, ncell, nops, sink, 7u);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(k_probe<MODE>, dim3(2048), dim3(256), 0, 0, tab, ncell, nops, sink, (uint32_t)r * 131u);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv)
{
    const uint64_t nops = 1ull << 27;   // 134M operations per launch
    const size_t sizes[] = {4ull << 20, 200ull << 20, 2048ull << 20};
    const char* names[] = {"load", "store", "amin_nr", "amin_r", "cas64", "cas64_row"};
    uint32_t* tab;
    uint32_t* sink;
    CK(hipMalloc(&tab, sizes[2]));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(tab, 0xFF, sizes[2]));
    for (size_t s : sizes) {
        const uint64_t ncell = s / 4;
        float ms[6];
        ms[0] = run<0>(tab, ncell, nops, sink, 5);
        ms[1] = run<1>(tab, ncell, nops, sink, 5);
        ms[2] = run<2>(tab, ncell, nops, sink, 5);
        ms[3] = run<3>(tab, ncell, nops, sink, 5);
        ms[4] = run<4>(tab, ncell / 2 * 2, nops, sink, 5);
        ms[5] = run<5>(tab, ncell, nops, sink, 5);
        for (int m = 0; m < 6; ++m) {
            const double ops = (m == 5) ? nops / 4.0 : (double)nops;
            printf("{\"table_mb\": %zu, \"mode\": \"%s\", \"ms\": %.3f, \"gops\": %.2f}\n", s >> 20, names[m], ms[m],
                   ops / (ms[m] * 1e-3) / 1e9);
        }
    }
    return 0;
}
