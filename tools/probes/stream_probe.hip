// Streaming-read probe for the Gram's access shape: 15 FP64 SoA columns of a 3M-row panel
// (600 x 5000), each lane owning RPL consecutive rows per tile, NBUF register buffers in
// flight per wave.  Measures the chip-wide read rate of each loop skeleton (HIP events).
// hipcc --offload-arch=gfx950 -O3 stream_probe.hip -o stream_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int NC = 15;

template <int RPL>
struct Vec;
template <>
struct Vec<1> {
    typedef double T;
};
template <>
struct Vec<2> {
    typedef double __attribute__((ext_vector_type(2))) T;
};

__device__ __forceinline__ double hsum(double v) { return v; }
__device__ __forceinline__ double hsum(double __attribute__((ext_vector_type(2))) v) { return v.x + v.y; }

// Each wave streams tiles [t_begin, t_end) of TR = 64 * RPL rows; tiles are laid out so
// that wave k of workgroup b takes a contiguous share (persistent) or the chunk's tiles
// w, w + 4, ... (chunked, one workgroup per chunk).
template <int RPL, int NBUF, bool PERSIST>
__global__ __launch_bounds__(256, 2) void stream_kernel(const double* __restrict__ cols, long long n,
                                                         long long stride, int chunk_rows,
                                                         double* out) {
    typedef typename Vec<RPL>::T V;
    constexpr int TR = 64 * RPL;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    long long t0, t1, tstep;
    long long ntile_total = (n + TR - 1) / TR;
    if (PERSIST) {
        const long long nw = (long long)gridDim.x * 4;
        const long long gw = (long long)blockIdx.x * 4 + w;
        t0 = ntile_total * gw / nw;
        t1 = ntile_total * (gw + 1) / nw;
        tstep = 1;
    } else {
        const long long r0 = (long long)blockIdx.x * chunk_rows;
        const long long c0 = r0 / TR;
        const long long c1 = (r0 + chunk_rows + TR - 1) / TR < ntile_total ? (r0 + chunk_rows + TR - 1) / TR
                                                                           : ntile_total;
        t0 = c0 + w;
        t1 = c1;
        tstep = 4;
    }
    V buf[NBUF][NC];
    double acc = 0.0;
    auto load = [&](V (&x)[NC], long long t) {
        long long tt = t < ntile_total ? t : ntile_total - 1;
        const double* p = cols + tt * TR + lane * RPL;
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] = *(const V*)(p + c * stride);
    };
    auto proc = [&](V (&x)[NC]) {
#pragma unroll
        for (int c = 0; c < NC; ++c) acc += hsum(x[c]);
    };
#pragma unroll
    for (int b = 0; b < NBUF - 1; ++b) load(buf[b], t0 + b * tstep);
    long long t = t0;
    while (t < t1) {
#pragma unroll
        for (int b = 0; b < NBUF; ++b) {
            load(buf[(b + NBUF - 1) % NBUF], t + (NBUF - 1) * tstep);
            proc(buf[b]);
            t += tstep;
            if (t >= t1) break;
        }
    }
    out[(long long)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int RPL, int NBUF, bool PERSIST>
void run(const char* name, const double* cols, long long n, int grid, int chunk_rows, double* out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((stream_kernel<RPL, NBUF, PERSIST>), dim3(grid), dim3(256), 0, 0, cols, n, n,
                           chunk_rows, out);
    const int reps = 20;
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((stream_kernel<RPL, NBUF, PERSIST>), dim3(grid), dim3(256), 0, 0, cols, n, n,
                           chunk_rows, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double gb = (double)n * NC * 8 / 1e9;
    printf("%-34s grid=%6d  %8.1f us  %7.2f TB/s\n", name, grid, ms * 1e3, gb / ms);
}

int main() {
    const long long n = 600LL * 5000;
    double* cols;
    double* out;
    hipMalloc(&cols, n * NC * 8);
    hipMalloc(&out, 1 << 24);
    hipMemset(cols, 0, n * NC * 8);
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int ch = 1280;
    const int nch = (int)((n + ch - 1) / ch);
    run<1, 2, false>("chunked rpl1 nbuf2 (1280 rows)", cols, n, nch, ch, out);
    run<1, 2, false>("chunked rpl1 nbuf2 (2560 rows)", cols, n, (int)((n + 2559) / 2560), 2560, out);
    run<2, 2, false>("chunked rpl2 nbuf2 (2560 rows)", cols, n, (int)((n + 2559) / 2560), 2560, out);
    for (int k : {1, 2, 3, 4}) {
        char nm[64];
        snprintf(nm, 64, "persist rpl1 nbuf2 x%d", k);
        run<1, 2, true>(nm, cols, n, ncu * k, 0, out);
        snprintf(nm, 64, "persist rpl1 nbuf3 x%d", k);
        run<1, 3, true>(nm, cols, n, ncu * k, 0, out);
        snprintf(nm, 64, "persist rpl2 nbuf2 x%d", k);
        run<2, 2, true>(nm, cols, n, ncu * k, 0, out);
    }
    hipFree(cols);
    hipFree(out);
    return 0;
}
