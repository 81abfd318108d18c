// Latency/throughput probe for v_mfma_f64_16x16x4_f64 and v_mfma_f64_4x4x4_4b_f64 on gfx950:
// cycles per MFMA (s_memtime, one wave alone on the chip and all CUs busy) for 1/2/4/8
// interleaved accumulator chains, plus the 4x4x4 lane layout (A, B, D index maps).
// hipcc --offload-arch=gfx950 -O3 mfma_f64_chains.hip -o mfma_f64_chains
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(64) void chains(double* out, long long* cyc, int iters) {
    const double a = 1.0 + threadIdx.x * 1e-9, b = 0.999;
    d4 c[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) c[k] = d4{0, 0, 0, 0};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8 / CH; ++r)
#pragma unroll
            for (int k = 0; k < CH; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int k = 0; k < CH; ++k) s += c[k].x + c[k].y + c[k].z + c[k].w;
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
__global__ __launch_bounds__(64) void chains4(double* out, long long* cyc, int iters) {
    const double a = 1.0 + threadIdx.x * 1e-9, b = 0.999;
    double c[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) c[k] = 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8 / CH; ++r)
#pragma unroll
            for (int k = 0; k < CH; ++k) c[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[k], 0, 0, 0);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int k = 0; k < CH; ++k) s += c[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// layout: A[lane] = 1 at one lane only, B = lane code; read which D entries change
__global__ void layout4(double* out, int hot) {
    const int l = threadIdx.x;
    const double av = l == hot ? 1.0 : 0.0;
    const double bv = 1000.0 + l;
    double d = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv, 0.0, 0, 0, 0);
    out[l] = d;
}

template <typename K>
void run(const char* name, K k, int blocks, int iters) {
    double* out;
    long long* cyc;
    hipMalloc(&out, sizeof(double) * blocks * 64);
    hipMalloc(&cyc, sizeof(long long) * blocks);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, cyc, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c0;
    hipMemcpy(&c0, cyc, sizeof(c0), hipMemcpyDeviceToHost);
    const double per = (double)c0 / (iters * 8.0);
    // wall: SIMD-seconds per instruction at the wall clock
    const double waves = blocks, inst = waves * iters * 8.0;
    const double simds = blocks < 1024 ? blocks : 1024;
    printf("%-34s blocks=%5d  memtime-cyc/MFMA(wave0)=%7.1f  wall ns/MFMA/SIMD=%7.2f\n", name, blocks,
           per, ms * 1e6 * simds / inst);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int blocks : {1, 1024, 2048}) {
        run("16x16x4 1 chain", chains<1>, blocks, 4096);
        run("16x16x4 2 chains", chains<2>, blocks, 4096);
        run("16x16x4 4 chains", chains<4>, blocks, 4096);
        run("16x16x4 8 chains", chains<8>, blocks, 4096);
        run("4x4x4 1 chain", chains4<1>, blocks, 4096);
        run("4x4x4 4 chains", chains4<4>, blocks, 4096);
        run("4x4x4 8 chains", chains4<8>, blocks, 4096);
    }
    // s_memtime ticks vs wall: one block, 4096*8 MFMAs
    double* out;
    hipMalloc(&out, 64 * sizeof(double));
    double h[64];
    for (int hot : {0, 1, 4, 5, 16, 17, 20}) {
        hipLaunchKernelGGL(layout4, dim3(1), dim3(64), 0, 0, out, hot);
        hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
        printf("4x4x4 A hot lane %2d ->", hot);
        for (int l = 0; l < 64; ++l)
            if (h[l] != 0.0) printf(" D[%d]=%g", l, h[l]);
        printf("\n");
    }
    return 0;
}
