// valu_peak.hip -- measures the integer VALU issue rate of gfx950 for the
// instruction mix of the SHA-256 kernels (v_alignbit_b32, v_bitop3_b32,
// v_add_u32), and the engine clock the chip holds under that load
// (s_memtime / s_memrealtime, MI355X_MICROARCH.md "DVFS give-back" item 6).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/valu_peak tools/valu_peak.hip
// Output: one JSON line.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHAINS 8
#define ITERS 4096

// 8 independent chains, each iteration 3 VALU ops per chain (alignbit,
// bitop3, add): 24 ops per iteration per lane.
__global__ __launch_bounds__(256) void valu_loop(uint32_t* out, uint32_t seed, uint64_t* clk) {
    uint32_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * (c + 1) ^ seed;
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < ITERS; ++i) {
        seed = __builtin_amdgcn_readfirstlane(seed + (uint32_t)i);
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            uint32_t r = __builtin_amdgcn_alignbit(x[c], x[c], 7);
            r = __builtin_amdgcn_bitop3_b32(r, x[c], seed, 0x96);
            x[c] = r + x[c];
        }
    }
    if (threadIdx.x == 0 && blockIdx.x < 1024) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc ^= x[c];
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keep live
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    uint32_t* out;
    uint64_t* clk;
    hipMalloc(&out, 1 << 20);
    hipMalloc(&clk, 1024 * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // grid: blocks per CU in {1, 2, 4, 8} (waves/SIMD = blocks per CU)
    printf("{\"cus\": %d, \"clock_khz\": %d, \"runs\": [", cus, prop.clockRate);
    for (int bpc = 1, first = 1; bpc <= 8; bpc *= 2, first = 0) {
        const int blocks = cus * bpc * 8;  // 8 rounds of full residency
        valu_loop<<<blocks, 256>>>(out, 1u, clk);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 3; ++r) valu_loop<<<blocks, 256>>>(out, (uint32_t)r, clk);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        uint64_t h[2048];
        hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
        double ratio = 0;
        int n = 0;
        for (int i = 0; i < 1024 && i < blocks; ++i)
            if (h[2 * i + 1]) {
                ratio += (double)h[2 * i] / (double)h[2 * i + 1];
                ++n;
            }
        const double ghz = n ? ratio / n * 0.1 : 0.0;  // memrealtime ticks at 100 MHz
        const double ops = 3.0 * blocks * 256.0 * ITERS * CHAINS * 3.0;
        printf("%s{\"waves_per_simd\": %d, \"tops\": %.3f, \"clock_ghz\": %.3f}", first ? "" : ", ", bpc,
               ops / (ms * 1e-3) / 1e12, ghz);
    }
    printf("]}\n");
    return 0;
}
