// probe_bw.hip — what HBM bandwidth does the refresh+score access pattern get?
//
// Standalone (no torch).  Allocates the C3 layout (T=16 planes of E=32M per
// field) and times access patterns with hipEvents:
//   copy16   : float4 stream copy (reference ceiling)
//   rd_soa   : wave-per-64-edges, read 4 f64 + 1 u8 per (t,e), reduce
//   rw_dense : same, write the 4 f64 back (x*0.97)
//   rw_sparse: same, write each f64 back with probability ~p (data-dependent)
//   rd_soa_t : thread-per-edge loop over topics (the naive shape), read only
// build: hipcc --offload-arch=gfx950 -O3 tools/probe_bw.hip -o tools/probe_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__global__ void k_copy16(const float4* __restrict__ a, float4* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

template <int MODE, int CHUNK>
__global__ __launch_bounds__(256) void k_soa(double* f0, double* f1, double* f2, double* f3, const uint8_t* fl,
                                             int64_t E, int T, double* sink, uint32_t pmask)
{
    const int lane = threadIdx.x & 63;
    const int64_t ntiles = E / 64;
    double acc = 0.0;
    for (int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); tile < ntiles; tile += (int64_t)gridDim.x * 4) {
        const int64_t e = tile * 64 + lane;
        for (int t0 = 0; t0 < T; t0 += CHUNK) {
            double a[CHUNK], b[CHUNK], c[CHUNK], d[CHUNK];
            uint8_t f[CHUNK];
#pragma unroll
            for (int j = 0; j < CHUNK; ++j) {
                const int64_t i = (int64_t)(t0 + j) * E + e;
                a[j] = f0[i]; b[j] = f1[i]; c[j] = f2[i]; d[j] = f3[i]; f[j] = fl[i];
            }
#pragma unroll
            for (int j = 0; j < CHUNK; ++j) {
                const int64_t i = (int64_t)(t0 + j) * E + e;
                acc += a[j] + b[j] + c[j] + d[j] + f[j];
                if (MODE == 1) { f0[i] = a[j] * 0.97; f1[i] = b[j] * 0.97; f2[i] = c[j] * 0.97; f3[i] = d[j] * 0.97; }
                if (MODE == 2) {
                    const uint32_t h = (uint32_t)(i * 2654435761u);
                    f0[i] = a[j] * 0.97;
                    if ((h & pmask) == 0) f1[i] = b[j] * 0.97;
                    if (((h >> 8) & pmask) == 0) f2[i] = c[j] * 0.97;
                    if (((h >> 16) & 31) == 0) f3[i] = d[j] * 0.97;
                }
            }
        }
    }
    if (acc == 12345.678) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_soa_thread(const double* f0, const double* f1, const double* f2,
                                                    const double* f3, const uint8_t* fl, int64_t E, int T,
                                                    double* sink)
{
    double acc = 0.0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x)
        for (int t = 0; t < T; ++t) {
            const int64_t i = (int64_t)t * E + e;
            acc += f0[i] + f1[i] + f2[i] + f3[i] + fl[i];
        }
    if (acc == 12345.678) sink[0] = acc;
}

int main(int argc, char** argv)
{
    const int64_t E = argc > 1 ? atoll(argv[1]) : 32000000;
    const int T = 16;
    const size_t n = (size_t)E * T;
    double *f0, *f1, *f2, *f3, *sink;
    uint8_t* fl;
    CK(hipMalloc(&f0, n * 8)); CK(hipMalloc(&f1, n * 8)); CK(hipMalloc(&f2, n * 8)); CK(hipMalloc(&f3, n * 8));
    CK(hipMalloc(&fl, n)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(f0, 0, n * 8)); CK(hipMemset(f1, 0, n * 8)); CK(hipMemset(f2, 0, n * 8)); CK(hipMemset(f3, 0, n * 8));
    CK(hipMemset(fl, 1, n));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto time = [&](const char* name, double bytes, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const size_t n4 = n * 8 / 16;
    time("copy16 (f0->f1, 16B/lane)", 2.0 * n * 8, [&] {
        hipLaunchKernelGGL(k_copy16, dim3(8192), dim3(256), 0, 0, (const float4*)f0, (float4*)f1, n4);
    });
    for (int g : {2048, 8192, 32768}) {
        char nm[64];
        snprintf(nm, sizeof nm, "rd_soa chunk4 grid%d", g);
        time(nm, 33.0 * n, [&] { hipLaunchKernelGGL((k_soa<0, 4>), dim3(g), dim3(256), 0, 0, f0, f1, f2, f3, fl, E, T, sink, 3u); });
    }
    time("rd_soa chunk8", 33.0 * n, [&] { hipLaunchKernelGGL((k_soa<0, 8>), dim3(8192), dim3(256), 0, 0, f0, f1, f2, f3, fl, E, T, sink, 3u); });
    time("rd_soa chunk16", 33.0 * n, [&] { hipLaunchKernelGGL((k_soa<0, 16>), dim3(8192), dim3(256), 0, 0, f0, f1, f2, f3, fl, E, T, sink, 3u); });
    time("rd_soa_thread", 33.0 * n, [&] { hipLaunchKernelGGL(k_soa_thread, dim3(16384), dim3(256), 0, 0, f0, f1, f2, f3, fl, E, T, sink); });
    time("rw_dense chunk4", 65.0 * n, [&] { hipLaunchKernelGGL((k_soa<1, 4>), dim3(8192), dim3(256), 0, 0, f0, f1, f2, f3, fl, E, T, sink, 3u); });
    time("rw_sparse chunk4 (compulsory bytes)", (33.0 + 8 + 2 + 2 + 0.25) * n,
         [&] { hipLaunchKernelGGL((k_soa<2, 4>), dim3(8192), dim3(256), 0, 0, f0, f1, f2, f3, fl, E, T, sink, 3u); });
    return 0;
}
