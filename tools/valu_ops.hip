// valu_ops.hip -- per-instruction VALU issue rate on gfx950 (wave64), so the
// SHA-256 kernels can pick the cheapest encodings.  Each kernel runs 8
// independent chains of ONE instruction (inline asm pins the encoding) with
// 8 waves per SIMD; reports lanes/clk/CU at the clock measured in-kernel.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/valu_ops tools/valu_ops.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

#define OP_KERNEL(NAME, ASM)                                                                      \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s, uint64_t* clk) {       \
        uint32_t x0 = threadIdx.x ^ s, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 9,         \
                 x5 = x0 * 11, x6 = x0 * 13, x7 = x0 * 15;                                        \
        const uint32_t y = threadIdx.x + s, z = threadIdx.x * s;                                  \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();        \
        for (int i = 0; i < ITERS; ++i) {                                                         \
            asm volatile(ASM : "+v"(x0) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x1) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x2) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x3) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x4) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x5) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x6) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x7) : "v"(y), "v"(z));                                        \
        }                                                                                         \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();        \
        if (threadIdx.x == 0 && blockIdx.x < 1024) {                                              \
            clk[2 * blockIdx.x] = t1 - t0;                                                        \
            clk[2 * blockIdx.x + 1] = r1 - r0;                                                    \
        }                                                                                         \
        const uint32_t acc = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                               \
        if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;                                            \
    }

OP_KERNEL(k_add_e32, "v_add_u32_e32 %0, %1, %0")
OP_KERNEL(k_add_e64, "v_add_u32_e64 %0, %1, %0")
OP_KERNEL(k_add3, "v_add3_u32 %0, %1, %2, %0")
OP_KERNEL(k_xor_e32, "v_xor_b32_e32 %0, %1, %0")
OP_KERNEL(k_xad, "v_xad_u32 %0, %1, %2, %0")
OP_KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %0, 7")
OP_KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
OP_KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
OP_KERNEL(k_lshr_e32, "v_lshrrev_b32_e32 %0, 3, %0")
OP_KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 3, %1")
OP_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
OP_KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
OP_KERNEL(k_mul_f32_e32, "v_mul_f32_e32 %0, %1, %0")
OP_KERNEL(k_mov_e32, "v_mov_b32_e32 %0, %1")

#define OP_KERNEL64(NAME, ASM)                                                                    \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s, uint64_t* clk) {       \
        uint64_t x0 = threadIdx.x ^ s, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 9,         \
                 x5 = x0 * 11, x6 = x0 * 13, x7 = x0 * 15;                                        \
        const uint32_t y = threadIdx.x + s, z = threadIdx.x * s;                                  \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();        \
        for (int i = 0; i < ITERS; ++i) {                                                         \
            asm volatile(ASM : "+v"(x0) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x1) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x2) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x3) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x4) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x5) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x6) : "v"(y), "v"(z));                                        \
            asm volatile(ASM : "+v"(x7) : "v"(y), "v"(z));                                        \
        }                                                                                         \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();        \
        if (threadIdx.x == 0 && blockIdx.x < 1024) {                                              \
            clk[2 * blockIdx.x] = t1 - t0;                                                        \
            clk[2 * blockIdx.x + 1] = r1 - r0;                                                    \
        }                                                                                         \
        const uint64_t acc = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                               \
        if (acc == 0x9e3779b9u) out[blockIdx.x] = (uint32_t)acc;                                  \
    }

OP_KERNEL64(k_lshr_b64, "v_lshrrev_b64 %0, 7, %0")
OP_KERNEL64(k_mov_b64, "v_mov_b64 %0, %0")
OP_KERNEL64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %0")
OP_KERNEL64(k_pk_mov_b32, "v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]")
OP_KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %0, 1")
OP_KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")
OP_KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
OP_KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
OP_KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
OP_KERNEL(k_sub_e32, "v_sub_u32_e32 %0, %1, %0")
OP_KERNEL(k_cndmask, "v_cndmask_b32_e64 %0, %0, %1, s[0:1]")
OP_KERNEL(k_add_lit, "v_add_u32_e32 %0, 0x428a2f98, %0")
OP_KERNEL(k_bitop3_lit, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8")
OP_KERNEL(k_lshlrev_e64, "v_lshlrev_b32_e64 %0, 7, %0")
OP_KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2")
OP_KERNEL(k_sdwa_xor, "v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")
// round 3: the opcodes valu_rates.py had classed by encoding only (ASSUMED)
OP_KERNEL(k_min_dpp, "v_min_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
OP_KERNEL(k_mov_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
OP_KERNEL(k_min3, "v_min3_u32 %0, %0, %1, %2")
OP_KERNEL(k_min_e32, "v_min_u32_e32 %0, %0, %1")
OP_KERNEL(k_and_e32, "v_and_b32_e32 %0, %0, %1")
OP_KERNEL(k_or_e32, "v_or_b32_e32 %0, %0, %1")
OP_KERNEL(k_lshl_e32, "v_lshlrev_b32_e32 %0, %1, %0")
OP_KERNEL(k_not_e32, "v_not_b32_e32 %0, %0")
OP_KERNEL(k_sub_e64, "v_sub_u32_e64 %0, %0, %1")
OP_KERNEL(k_cnd_e32, "v_cndmask_b32_e32 %0, %1, %0, vcc")
OP_KERNEL(k_cmp_e32, "v_cmp_lt_u32_e32 vcc, %0, %1")
OP_KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
OP_KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
OP_KERNEL(k_add_lshl, "v_add_lshl_u32 %0, %0, %1, 3")
OP_KERNEL(k_lshr_e64, "v_lshrrev_b32_e64 %0, 7, %0")

typedef void (*kfn)(uint32_t*, uint32_t, uint64_t*);

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    uint32_t* out;
    uint64_t* clk;
    (void)hipMalloc(&out, 1 << 20);
    (void)hipMalloc(&clk, 1024 * 16);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    struct {
        const char* name;
        kfn f;
    } ks[] = {{"v_add_u32_e32", k_add_e32}, {"v_add_u32_e64", k_add_e64}, {"v_add3_u32", k_add3},
              {"v_xor_b32_e32", k_xor_e32}, {"v_xad_u32", k_xad},         {"v_alignbit_b32", k_alignbit},
              {"v_bitop3_b32", k_bitop3},   {"v_bfi_b32", k_bfi},         {"v_lshrrev_b32_e32", k_lshr_e32},
              {"v_lshl_or_b32", k_lshl_or}, {"v_perm_b32", k_perm},       {"v_fma_f32", k_fma_f32},
              {"v_mul_f32_e32", k_mul_f32_e32}, {"v_mov_b32_e32", k_mov_e32},
              {"v_lshrrev_b64", k_lshr_b64}, {"v_mov_b64", k_mov_b64}, {"v_pk_add_f32", k_pk_add_f32},
              {"v_pk_mov_b32", k_pk_mov_b32}, {"v_alignbyte_b32", k_alignbyte}, {"v_or3_b32", k_or3},
              {"v_and_or_b32", k_and_or}, {"v_lshl_add_u32", k_lshl_add}, {"v_pk_add_u16", k_pk_add_u16},
              {"v_sub_u32_e32", k_sub_e32}, {"v_cndmask_b32_e64", k_cndmask}, {"v_add_u32_e32+lit", k_add_lit},
              {"v_bitop3_b32(maj)", k_bitop3_lit}, {"v_lshlrev_b32_e64", k_lshlrev_e64},
              {"v_mad_u32_u24", k_mad_u24}, {"v_xor_b32_sdwa(w1)", k_sdwa_xor},
              {"v_min_u32_dpp", k_min_dpp}, {"v_mov_b32_dpp", k_mov_dpp}, {"v_min3_u32", k_min3},
              {"v_min_u32_e32", k_min_e32}, {"v_and_b32_e32", k_and_e32}, {"v_or_b32_e32", k_or_e32},
              {"v_lshlrev_b32_e32", k_lshl_e32}, {"v_not_b32_e32", k_not_e32}, {"v_sub_u32_e64", k_sub_e64},
              {"v_cndmask_b32_e32", k_cnd_e32}, {"v_cmp_lt_u32_e32", k_cmp_e32}, {"v_mul_lo_u32", k_mul_lo},
              {"v_mul_hi_u32", k_mul_hi}, {"v_add_lshl_u32", k_add_lshl}, {"v_lshrrev_b32_e64", k_lshr_e64}};
    printf("{\"cus\": %d, \"ops\": {", cus);
    const int nk = sizeof ks / sizeof ks[0];
    for (int w = 0; w < 2; ++w) {
        const int wps = w ? 8 : 4;  // waves per SIMD
        const int blocks = cus * wps * 4;
        for (int k = 0; k < nk; ++k) {
            hipLaunchKernelGGL(ks[k].f, dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(a);
            for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(ks[k].f, dim3(blocks), dim3(256), 0, 0, out, 2u, clk);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            uint64_t h[2048];
            (void)hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
            double ratio = 0;
            int n = 0;
            for (int i = 0; i < 1024 && i < blocks; ++i)
                if (h[2 * i + 1]) {
                    ratio += (double)h[2 * i] / (double)h[2 * i + 1];
                    ++n;
                }
            const double ghz = n ? ratio / n * 0.1 : 0.0;
            const double lane_ops = 2.0 * blocks * 256.0 * ITERS * 8.0;
            const double per_clk_cu = lane_ops / (ms * 1e-3) / (ghz * 1e9) / cus;
            printf("%s\"%s@%dw\": {\"lanes_per_clk_cu\": %.1f, \"tops\": %.2f, \"ghz\": %.3f}",
                   (w == 0 && k == 0) ? "" : ", ", ks[k].name, wps, per_clk_cu, lane_ops / (ms * 1e-3) / 1e12, ghz);
        }
    }
    printf("}}\n");
    return 0;
}
