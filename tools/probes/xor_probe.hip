// Probe: lane-xor exchanges without LDS (DPP row_ror / quad_perm, permlane16/32_swap) vs
// __shfl_xor, for j = 1..32.  Prints one line per distance.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int J>
__device__ __forceinline__ unsigned xorx(unsigned x) {
    const int lane = __lane_id();
    if constexpr (J == 1) return __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    if constexpr (J == 2) return __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    if constexpr (J == 4) {
        const unsigned t = __builtin_amdgcn_update_dpp(x, x, 0x12C, 0xF, 0x5, false);      // row_ror:12, banks 0,2
        return __builtin_amdgcn_update_dpp(t, x, 0x124, 0xF, 0xA, false);                 // row_ror:4, banks 1,3
    }
    if constexpr (J == 8) return __builtin_amdgcn_update_dpp(x, x, 0x128, 0xF, 0xF, false);  // row_ror:8
    if constexpr (J == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16) ? r[0] : r[1];
    }
    if constexpr (J == 32) {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
    return 0;
}

template <int J>
__global__ void probe(unsigned* out) {
    const unsigned x = __lane_id() * 7u + 3u;
    out[threadIdx.x] = (xorx<J>(x) == (unsigned)__shfl_xor((int)x, J, 64)) ? 1u : 0u;
}

int main() {
    unsigned* d;
    unsigned h[64];
    hipMalloc(&d, 64 * 4);
    auto run = [&](auto kern, int j) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d);
        hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
        int ok = 0;
        for (int i = 0; i < 64; ++i) ok += h[i];
        printf("xor %2d: %d/64 lanes match\n", j, ok);
    };
    run(probe<1>, 1);
    run(probe<2>, 2);
    run(probe<4>, 4);
    run(probe<8>, 8);
    run(probe<16>, 16);
    run(probe<32>, 32);
    return 0;
}
