"""Generate tools/valu_pair.hip: which full-rate VALU ops co-issue beside the
half-rate ones on gfx950.

PMC of fast_search<4,0> (profiles/r02c_bench.json): the VALU is busy every
quad-cycle (VALUBusy 1.04) yet only 5.3% of quad-cycles issue two VALU
instructions (SQ_ACTIVE_INST_VALU2), so the loop runs 3.83 cycles per
instruction against 3.17 if every full-rate op shared a quad-cycle.  The
r01 mixes (gen_valu_mix.py) showed that a VOP2 add after a half-rate op never
pairs (HF 4.0) while a VOP3 v_bitop3 sometimes does (HB 3.68, HBB 3.40).
These patterns separate encoding (VOP2 e32 / VOP3 e64), opcode and dependency.

Each pattern is one opaque asm block over 8 independent chains (instruction i
on chain i mod 8) unless its name ends in _DEP, where each group of the
pattern runs on one chain (every instruction reads the previous one)."""
H = "v_alignbit_b32 {x}, {x}, {x}, 7"
A3 = "v_add3_u32 {x}, {x}, {y}, {x}"
F = "v_add_u32_e32 {x}, {y}, {x}"
F3 = "v_add_u32_e64 {x}, {y}, {x}"
X = "v_xor_b32_e32 {x}, {y}, {x}"
X3 = "v_xor_b32_e64 {x}, {y}, {x}"
S = "v_lshrrev_b32_e32 {x}, 3, {x}"
S3 = "v_lshrrev_b32_e64 {x}, 3, {x}"
B = "v_bitop3_b32 {x}, {x}, {y}, {x} bitop3:0x96"
B2 = "v_bitop3_b32 {x}, {x}, {y}, {y} bitop3:0xca"
PATTERNS = {
    "H": [H], "F": [F], "F3": [F3], "X3": [X3], "S": [S], "S3": [S3], "B": [B], "B2": [B2],
    "HF": [H, F], "HF3": [H, F3], "HX3": [H, X3], "HS": [H, S], "HS3": [H, S3], "HB": [H, B], "HB2": [H, B2],
    "HBB": [H, B, B], "HF3F3": [H, F3, F3], "HBF3": [H, B, F3], "HB2B": [H, B2, B],
    "BF": [B, F], "BF3": [B, F3], "F3X3": [F3, X3], "FF3": [F, F3],
    "A3F3": [A3, F3], "A3B": [A3, B],
    # the per-nonce loop's multiset per 14 instructions: 6 alignbit, 2.3 add3, 3.6 bitop3, 1.3 add, 0.85 shift
    "ROUND": [H, H, H, B, B, H, H, H, A3, B, B, A3, A3, F],
    "ROUND_F3": [H, H, H, B, B, H, H, H, A3, B, B, A3, A3, F3],
    "ROUND_HB": [H, B, H, B, H, B, H, B, H, A3, H, A3, A3, F3],
    # an add3 split into two full-rate adds
    "ROUND_SPLIT": [H, H, H, B, B, H, H, H, F3, F3, B, B, F3, F3, A3, F3],
    # dependent pairs: H then B reading H's result (the Sigma shape)
    "HB_DEP": [H, B], "HBB_DEP": [H, B, B], "HF3_DEP": [H, F3],
}
# r02o: priority phases.  s_setprio is a scalar instruction (no VALU slot).  A wave entering a run
# of full-rate ops raises its priority, so the arbiter prefers waves whose next VALU op can pair
P3, P0 = "s_setprio 3", "s_setprio 0"
PATTERNS.update({
    "H4F4": [H] * 4 + [F] * 4, "H4F4_PRIO": [P0] + [H] * 4 + [P3] + [F] * 4,
    "H6F4": [H] * 6 + [F] * 4, "H6F4_PRIO": [P0] + [H] * 6 + [P3] + [F] * 4,
    "H4B4": [H] * 4 + [B] * 4, "H4B4_PRIO": [P0] + [H] * 4 + [P3] + [B] * 4,
    "H8F8": [H] * 8 + [F] * 8, "H8F8_PRIO": [P0] + [H] * 8 + [P3] + [F] * 8,
    "H4F4_PRIOINV": [P3] + [H] * 4 + [P0] + [F] * 4,
    "H2F2_PRIO": [P0] + [H] * 2 + [P3] + [F] * 2,
    "H9F5_PRIO": [P0] + [H] * 9 + [P3] + [B] * 4 + [F],
    # r02p: priority on the HALF-rate phase (the wave about to issue full-rate ops yields)
    "H4B4_PRIOINV": [P3] + [H] * 4 + [P0] + [B] * 4,
    "H6F4_PRIOINV": [P3] + [H] * 6 + [P0] + [F] * 4,
    "H2F2_PRIOINV": [P3] + [H] * 2 + [P0] + [F] * 2,
    "HF_PRIOINV": [P3, H, P0, F],
    "HB_PRIOINV": [P3, H, P0, B],
    "H9F5_PRIOINV": [P3] + [H] * 9 + [P0] + [B] * 4 + [F],
    "H4F4_PRIOINV1": ["s_setprio 1"] + [H] * 4 + [P0] + [F] * 4,
    "H4A3F4_PRIOINV": [P3] + [H, A3, H, A3] + [P0] + [F] * 4,
    "ROUND_PRIOINV": [P3, H, H, H, P0, B, B, P3, H, H, H, A3, P0, B, B, P3, A3, A3, P0, F],
    "ROUND_GRP_PRIOINV": [P3, H, H, H, H, H, H, A3, A3, A3, P0, B, B, B, B, F],
    "F4H4_PRIOINV": [P0] + [F] * 4 + [P3] + [H] * 4,
})
DEP = {"HB_DEP", "HBB_DEP", "HF3_DEP"}
# r02h: loop-body size (instruction-fetch footprint): the same stream unrolled to ~1K / 2.5K / 5K
# instructions per loop iteration (the per-nonce loop is 1,196 instructions, ~8.8 KB)
SIZES = {}
for base, n in (("ROUND", 10), ("ROUND", 20), ("ROUND", 40), ("B", 8), ("B", 20), ("F", 20), ("HB", 20)):
    PATTERNS[f"{base}_x{n}"] = PATTERNS[base]
    SIZES[f"{base}_x{n}"] = n
ONLY = set(__import__("os").environ.get("VALU_PAIR_ONLY", "").split(",")) - {""}
if ONLY:
    PATTERNS = {k: v for k, v in PATTERNS.items() if k in ONLY or k.split("_x")[0] in ONLY and k in SIZES}


def lines_of(name, seq):
    reps = max(8, 128 // len(seq)) * SIZES.get(name, 1)
    out = []
    idx = 0
    for r in range(reps):
        for k, ins in enumerate(seq):
            if ins.startswith("s_"):
                out.append(ins)
                continue
            c = (idx // len(seq)) % 8 if name in DEP else idx % 8
            idx += 1
            out.append(ins.format(x="%" + str(c), y="%8"))
    return out


body = []
kernels = []
for name, seq in PATTERNS.items():
    lines = lines_of(name, seq)
    asm = "\\n\\t".join(lines)
    kernels.append((name, sum(1 for l in lines if not l.startswith("s_"))))
    body.append(f'''
__global__ __launch_bounds__(256) void k_{name}(uint32_t* out, uint32_t s, uint64_t* clk) {{
    uint32_t x0 = threadIdx.x ^ s, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 9, x5 = x0 * 11,
             x6 = x0 * 13, x7 = x0 * 15;
    const uint32_t y = threadIdx.x + s;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i)
        asm volatile("{asm}" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6),
                     "+v"(x7) : "v"(y));
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 4096) {{ clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }}
    const uint32_t acc = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}}''')
src = '''// GENERATED by tools/gen_valu_pair.py -- co-issue of full-rate VALU ops beside half-rate ones, gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ITERS 64
''' + "\n".join(body) + '''
typedef void (*kfn)(uint32_t*, uint32_t, uint64_t*);
int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    uint32_t* out; uint64_t* clk;
    (void)hipMalloc(&out, 1 << 20); (void)hipMalloc(&clk, 4096 * 16);
    struct { const char* name; kfn f; int nins; } ks[] = {
''' + ",\n".join(f'        {{"{n}", k_{n}, {ni}}}' for n, ni in kernels) + '''};
    printf("{\\"cus\\": %d, \\"patterns\\": {", cus);
    const int nk = sizeof ks / sizeof ks[0];
    const int wps_list[] = {2, 6, 8};  // resident waves per SIMD (256-thread blocks: one wave per SIMD each)
    for (int wi = 0, first = 1; wi < 3; ++wi) {
        const int wps = wps_list[wi];
        const int blocks = cus * wps;
        for (int k = 0; k < nk; ++k, first = 0) {
            hipLaunchKernelGGL(ks[k].f, dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
            (void)hipDeviceSynchronize();
            hipEvent_t ea, eb; (void)hipEventCreate(&ea); (void)hipEventCreate(&eb);
            (void)hipEventRecord(ea);
            hipLaunchKernelGGL(ks[k].f, dim3(blocks), dim3(256), 0, 0, out, 2u, clk);
            (void)hipEventRecord(eb); (void)hipEventSynchronize(eb);
            float ms = 0; (void)hipEventElapsedTime(&ms, ea, eb);
            static uint64_t h[8192];
            (void)hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
            double cyc = 0, rt = 0; int n = 0;
            for (int i = 0; i < 4096 && i < blocks; ++i) if (h[2 * i + 1]) { cyc += (double)h[2 * i]; rt += (double)h[2 * i + 1]; ++n; }
            const double ghz = cyc / rt * 0.1;  // memtime ticks per 10 ns memrealtime tick
            // SIMD cycles per wave-instruction over the whole kernel (event time)
            const double simd_cpi = (ms * 1e-3) * ghz * 1e9 * cus * 4 / ((double)blocks * 4 * ITERS * ks[k].nins);
            // per-wave view: a wave's own loop cycles / (its instructions x waves sharing the SIMD)
            const double wave_cpi = (cyc / n) / ((double)ITERS * ks[k].nins * wps);
            printf("%s\\"%s@%d\\": {\\"simd_cyc_per_instr\\": %.3f, \\"wave_cyc_per_instr\\": %.3f, \\"ghz\\": %.3f, \\"nins\\": %d}",
                   first ? "" : ", ", ks[k].name, wps, simd_cpi, wave_cpi, ghz, ks[k].nins);
            (void)hipEventDestroy(ea); (void)hipEventDestroy(eb);
        }
    }
    printf("}}\\n");
    return 0;
}
'''
open("tools/valu_pair.hip", "w").write(src)
