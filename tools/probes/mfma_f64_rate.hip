// Throughput probe: FP64 MFMA 16x16x4 and 4x4x4 vs FP64 VALU FMA on gfx950.
// hipcc --offload-arch=gfx950 -O3 mfma_f64_rate.hip -o mfma_f64_rate && ./mfma_f64_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(double* out, int iters, double seed) {
    double a = seed + threadIdx.x * 1e-3, b = seed * 0.5;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double v0 = a, v1 = b, v2 = a * b, v3 = a + b;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
        } else if (MODE == 1) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        } else if (MODE == 2) {
            c0.x = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0.x, 0, 0, 0);
            c0.y = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0.y, 0, 0, 0);
            c0.z = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0.z, 0, 0, 0);
            c0.w = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0.w, 0, 0, 0);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v0 = fma(v0, a, b);
                v1 = fma(v1, a, b);
                v2 = fma(v2, a, b);
                v3 = fma(v3, a, b);
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0.x + c1.y + c2.z + c3.w + v0 + v1 + v2 + v3;
}

template <int MODE>
void run(const char* name, double flops_per_iter_per_wave) {
    const int blocks = 256 * 8, iters = 4096;
    double* out;
    (void)hipMalloc(&out, sizeof(double) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    probe<MODE><<<blocks, 256>>>(out, 16, 1.0);
    (void)hipEventRecord(e0);
    probe<MODE><<<blocks, 256>>>(out, iters, 1.0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0;
    const double tf = waves * iters * flops_per_iter_per_wave / (ms * 1e-3) / 1e12;
    // cycles per instruction per SIMD at 2.4 GHz: SIMD-seconds / instructions
    const double inst = waves * iters * 4.0;
    const double cyc = (ms * 1e-3) * 2.4e9 * 1024.0 / inst;
    printf("%-28s %8.3f ms  %7.2f TFLOP/s  %6.1f cyc/inst/SIMD@2.4GHz\n", name, ms, tf, cyc);
    (void)hipFree(out);
}

int main() {
    run<0>("mfma_f64_16x16x4 indep", 4 * 16 * 16 * 4 * 2.0);
    run<1>("mfma_f64_16x16x4 dependent", 4 * 16 * 16 * 4 * 2.0);
    run<2>("mfma_f64_4x4x4 (16 blk)", 4 * 4 * 4 * 4 * 16 * 2.0);
    run<3>("v_fma_f64 (wave64)", 16 * 64 * 2.0);
    return 0;
}
