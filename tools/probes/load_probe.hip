// Load-shape probe for the long select's unit read (a 20,000-value high-word month column per
// 512-thread workgroup, one workgroup per unit): 4-byte vs 16-byte buffer loads per lane, with
// 80 VGPRs' occupancy (3 workgroups per CU); and what a misaligned 16-byte load straddling
// the descriptor's range returns.  Each workgroup reduces its
// words (min / max / count, one block sum) so the loads are live.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/load_probe tools/probes/load_probe.hip && tools/probes/load_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

constexpr int LT = 512;

template <int W>   // W dwords per load (1 or 4); 40 words per thread
__global__ __launch_bounds__(LT, 6) void probe(const uint32_t* hp, int L, int64_t stride, uint32_t* out) {
    constexpr int NV = 40 / W;
    const int u = blockIdx.x;
    const uint32_t* base = hp + (int64_t)u * stride;
    uint32_t mn = 0xFFFFFFFFu, mx = 0;
    int cnt = 0;
    if constexpr (W == 1) {
        uint32_t h[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int rem = L - v * LT;
            const int nrec = rem > 0 ? (rem < LT ? rem : LT) * 4 : 0;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(base + (rem > 0 ? v * LT : 0)), 0, nrec, 0x00020000);
            h[v] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, threadIdx.x * 4u, 0, 0);
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            mn = min(mn, h[v]);
            mx = max(mx, h[v]);
            cnt += (int)__popcll(__ballot(h[v] < 0x7FF00000u));
        }
    } else {
        uint32_t h[NV][4];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int rem = L - v * LT * 4;
            const int nrec = rem > 0 ? (rem < LT * 4 ? rem : LT * 4) * 4 : 0;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(base + (rem > 0 ? v * LT * 4 : 0)), 0, nrec, 0x00020000);
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16u, 0, 0);
            h[v][0] = q[0];
            h[v][1] = q[1];
            h[v][2] = q[2];
            h[v][3] = q[3];
        }
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                mn = min(mn, h[v][j]);
                mx = max(mx, h[v][j]);
                cnt += (int)__popcll(__ballot(h[v][j] < 0x7FF00000u));
            }
    }
    __shared__ uint32_t red[3][LT / 64];
    const int w = threadIdx.x / 64;
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = mn;
        red[1][w] = mx;
        red[2][w] = (uint32_t)cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = red[0][0], b = red[1][0], c = red[2][0];
        for (int q = 1; q < LT / 64; ++q) {
            a = min(a, red[0][q]);
            b = max(b, red[1][q]);
            c += red[2][q];
        }
        out[3 * u] = a;
        out[3 * u + 1] = b;
        out[3 * u + 2] = c;
    }
}

// Semantics check: one wave loads 16 B per lane from a base 1 word past 16-B alignment with a
// range of 4 * 61 bytes: lanes 0..14 are in range, lane 15's four dwords straddle the end.
__global__ void semantics(const uint32_t* buf, uint32_t* out) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(buf + 1), 0, 4 * 61, 0x00020000);
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16u, 0, 0);
    for (int j = 0; j < 4; ++j) out[threadIdx.x * 4 + j] = q[j];
}

int main() {
    {
        uint32_t *b, *o;
        hipMalloc(&b, 4096);
        hipMalloc(&o, 4096);
        std::vector<uint32_t> h(1024);
        for (int i = 0; i < 1024; ++i) h[i] = 1000 + i;
        hipMemcpy(b, h.data(), 4096, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(semantics, dim3(1), dim3(64), 0, 0, b, o);
        hipMemcpy(h.data(), o, 4096, hipMemcpyDeviceToHost);
        printf("semantics (expect 1001.. for words 0..60, 0 past):");
        for (int i = 52; i < 68; ++i) printf(" %u", h[i]);
        printf("\n");
        hipFree(b);
        hipFree(o);
    }
    const int L = 20000, units = 15000;
    const int64_t stride = 20000;
    uint32_t *hp, *out;
    hipMalloc(&hp, (size_t)units * stride * 4);
    hipMalloc(&out, (size_t)units * 3 * 4);
    hipMemset(hp, 0x3F, (size_t)units * stride * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* tag, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        std::vector<float> ts;
        for (int r = 0; r < 9; ++r) {
            hipEventRecord(e0, 0);
            launch();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double ms = ts[ts.size() / 2];
        printf("%-8s %.3f ms  %.0f GB/s\n", tag, ms, (double)units * L * 4 / (ms * 1e-3) / 1e9);
    };
    run("dword", [&] { hipLaunchKernelGGL(probe<1>, dim3(units), dim3(LT), 0, 0, hp, L, stride, out); });
    run("dwordx4", [&] { hipLaunchKernelGGL(probe<4>, dim3(units), dim3(LT), 0, 0, hp, L, stride, out); });
    run("dword", [&] { hipLaunchKernelGGL(probe<1>, dim3(units), dim3(LT), 0, 0, hp, L, stride, out); });
    run("dwordx4", [&] { hipLaunchKernelGGL(probe<4>, dim3(units), dim3(LT), 0, 0, hp, L, stride, out); });
    hipFree(hp);
    hipFree(out);
    return 0;
}
