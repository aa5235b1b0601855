// valu_energy.hip -- what one VALU instruction class costs in energy on gfx950 at the power limit
// (price the instructions of the fast kernel's per-nonce loop in joules).
//
// Each kernel keeps every SIMD of the chip at 8 waves, each wave running ONE instruction class
// (inline asm pins the encoding) over 8 independent register chains, 64 instructions per
// iteration, between two absolute times of the 100 MHz counter (s_memrealtime) that the host
// derives from a timestamp kernel: every wave sleeps until the start time, so all of them are
// resident and start together (a wave launched into a SIMD whose older waves already saturate the
// VALU would otherwise wait for them: a time-per-wave loop then runs in generations), and runs its
// stream until the end time.  Every wave records its iterations, its shader cycles and 100 MHz
// ticks over the stream, and its XCD; the host (tools/energy_probe.py) reads the socket's energy
// counter inside [start, end] while the kernel runs and turns the counts into wave-instructions per
// second and the clock the chip held.
//
// The operands toggle like the SHA-256 loop's: rotations of a running value, sums and three-way
// xors with per-lane values.  Results go to a buffer of their own by vector stores (lane 0 of
// each wave); nothing else is written.
//
// C-ABI (build/libvaluenergy.so, loaded with ctypes; measurement only):
//   ve_kinds()                                        number of probe kinds
//   ve_name(kind)                                     its name
//   ve_valu_per_iter(kind), ve_salu_per_iter(kind)    instructions per wave-iteration
//   ve_start(dev, kind, delay_s, seconds, nwg)        launch nwg workgroups of 256 threads on
//                                                     device dev, their stream from delay_s after
//                                                     the call for seconds; returns at once
//   ve_wait(dev, out, nwg)                            wait for it; out[4*w..4*w+3] = {iterations,
//                                                     cycles, 100 MHz ticks, xcc} of wave w
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kXccIdReg = 20 | (3 << 11);  // s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4)

#define CH8(A0, A1, A2, A3, A4, A5, A6, A7)                                                     \
    asm volatile(A0 : "+v"(x0) : "v"(y), "v"(z));                                             \
    asm volatile(A1 : "+v"(x1) : "v"(y), "v"(z));                                             \
    asm volatile(A2 : "+v"(x2) : "v"(y), "v"(z));                                             \
    asm volatile(A3 : "+v"(x3) : "v"(y), "v"(z));                                             \
    asm volatile(A4 : "+v"(x4) : "v"(y), "v"(z));                                             \
    asm volatile(A5 : "+v"(x5) : "v"(y), "v"(z));                                             \
    asm volatile(A6 : "+v"(x6) : "v"(y), "v"(z));                                             \
    asm volatile(A7 : "+v"(x7) : "v"(y), "v"(z));
#define SAME8(A) CH8(A, A, A, A, A, A, A, A)
#define X8(B) B B B B B B B B

#define ALIGNBIT "v_alignbit_b32 %0, %0, %0, 7"
#define ADD3 "v_add3_u32 %0, %1, %2, %0"
#define BITOP3 "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96"
#define ADD "v_add_u32_e32 %0, %1, %0"
#define CH "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca"
#define MAJ "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8"
#define LSHR "v_lshrrev_b32_e32 %0, 3, %0"
#define PRIO_H "s_setprio 3\n\t" ALIGNBIT
#define PRIO_F "s_setprio 0\n\t" ADD
#define PRIO_FB "s_setprio 0\n\t" BITOP3

struct Kind {
    const char* name;
    int valu, salu;  // per wave-iteration (the loop's own compare and branch not counted)
};
constexpr Kind kKinds[] = {
    {"sleep", 0, 1},           // waves resident, s_sleep only: the chip's floor with a kernel up
    {"alignbit", 64, 0},       // half rate
    {"add3", 64, 0},           // half rate
    {"bitop3", 64, 0},         // full rate (xor3)
    {"add", 64, 0},            // full rate
    {"setprio", 0, 64},        // scalar: the issue-priority markers alone
    {"h4f4_prio", 64, 16},     // 4 alignbit + 4 add with the product's markers (pairs issue)
    {"h4b4_prio", 64, 16},     // 4 alignbit + 4 bitop3 with markers
    {"h4f4", 64, 0},           // the h4f4_prio stream without the markers
    {"seg", 64, 0},            // class-segregated waves: even waves alignbit only, odd waves add only
    {"bitop3_ch", 64, 0},      // bitop3:0xCA, SHA-256's Ch
    {"bitop3_maj", 64, 0},     // bitop3:0xE8, SHA-256's Maj
    {"lshr", 64, 0},           // v_lshrrev_b32 (the schedule's shifts)
};
constexpr int kNumKinds = sizeof(kKinds) / sizeof(kKinds[0]);

__global__ void realtime_now(uint64_t* __restrict__ out) {
    if (threadIdx.x == 0) out[0] = __builtin_amdgcn_s_memrealtime();
}

template <int KIND>
__global__ __launch_bounds__(256) void valu_energy(uint64_t* __restrict__ out, uint32_t s, uint64_t r_start,
                                                   uint64_t r_end) {
    uint32_t x0 = (threadIdx.x * 0x9e3779b9u) ^ s, x1 = x0 * 3u + 1u, x2 = x0 * 5u + 7u, x3 = x0 * 7u + 11u,
             x4 = x0 * 9u + 13u, x5 = x0 * 11u + 17u, x6 = x0 * 13u + 19u, x7 = x0 * 15u + 23u;
    const uint32_t y = (threadIdx.x + s) * 0x85ebca6bu, z = (threadIdx.x ^ 0x5bd1e995u) * 0xc2b2ae35u;
    uint64_t r = __builtin_amdgcn_s_memrealtime();
    while (r < r_start) {  // every wave resident and asleep until the common start
        __builtin_amdgcn_s_sleep(127);
        r = __builtin_amdgcn_s_memrealtime();
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = r;
    uint64_t it = 0;
    while (r < r_end) {
        if constexpr (KIND == 0) {
            __builtin_amdgcn_s_sleep(8);
        } else if constexpr (KIND == 1) {
            X8(SAME8(ALIGNBIT))
        } else if constexpr (KIND == 2) {
            X8(SAME8(ADD3))
        } else if constexpr (KIND == 3) {
            X8(SAME8(BITOP3))
        } else if constexpr (KIND == 4) {
            X8(SAME8(ADD))
        } else if constexpr (KIND == 5) {
            X8(asm volatile("s_setprio 0\n\ts_setprio 0\n\ts_setprio 0\n\ts_setprio 0\n\t"
                            "s_setprio 0\n\ts_setprio 0\n\ts_setprio 0\n\ts_setprio 0");)
        } else if constexpr (KIND == 6) {
            X8(CH8(PRIO_H, ALIGNBIT, ALIGNBIT, ALIGNBIT, PRIO_F, ADD, ADD, ADD))
        } else if constexpr (KIND == 7) {
            X8(CH8(PRIO_H, ALIGNBIT, ALIGNBIT, ALIGNBIT, PRIO_FB, BITOP3, BITOP3, BITOP3))
        } else if constexpr (KIND == 8) {
            X8(CH8(ALIGNBIT, ALIGNBIT, ALIGNBIT, ALIGNBIT, ADD, ADD, ADD, ADD))
        } else if constexpr (KIND == 9) {
            if ((__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6) & 1u) {
                X8(SAME8(ADD))
            } else {
                X8(SAME8(ALIGNBIT))
            }
        } else if constexpr (KIND == 10) {
            X8(SAME8(CH))
        } else if constexpr (KIND == 11) {
            X8(SAME8(MAJ))
        } else {
            X8(SAME8(LSHR))
        }
        ++it;
        r = __builtin_amdgcn_s_memrealtime();
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if constexpr (KIND == 5 || KIND == 6 || KIND == 7) __builtin_amdgcn_s_setprio(0);
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(kXccIdReg);
    const uint32_t acc = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if ((threadIdx.x & 63) < 4) {
        // the chains' value rides in the xcc word's upper half, so the compiler keeps every chain
        const uint64_t v[4] = {it, t1 - t0, r - r0, (uint64_t)xcc | ((uint64_t)(acc & 0xffffu) << 32)};
        out[4 * wave + (threadIdx.x & 63)] = v[threadIdx.x & 63];
    }
}

using KernelFn = void (*)(uint64_t*, uint32_t, uint64_t, uint64_t);
constexpr KernelFn kFns[] = {valu_energy<0>, valu_energy<1>, valu_energy<2>, valu_energy<3>, valu_energy<4>,
                             valu_energy<5>, valu_energy<6>, valu_energy<7>, valu_energy<8>, valu_energy<9>,
                             valu_energy<10>, valu_energy<11>, valu_energy<12>};
static_assert(sizeof(kFns) / sizeof(kFns[0]) == kNumKinds, "one kernel per kind");

}  // namespace

extern "C" int ve_kinds() { return kNumKinds; }
extern "C" const char* ve_name(int k) { return k >= 0 && k < kNumKinds ? kKinds[k].name : nullptr; }
extern "C" int ve_valu_per_iter(int k) { return k >= 0 && k < kNumKinds ? kKinds[k].valu : -1; }
extern "C" int ve_salu_per_iter(int k) { return k >= 0 && k < kNumKinds ? kKinds[k].salu : -1; }

constexpr int kMaxDevices = 64;
struct Slot {
    uint64_t* out = nullptr;  // non-null while a probe is outstanding
    int nwg = 0;
};
Slot g_slot[kMaxDevices];

extern "C" int ve_start(int dev, int kind, double delay_s, double seconds, int nwg) {
    if (dev < 0 || dev >= kMaxDevices || g_slot[dev].out) return -1;
    if (kind < 0 || kind >= kNumKinds || nwg < 1 || nwg > 65536 || !(seconds > 0 && seconds <= 30) ||
        !(delay_s >= 0 && delay_s <= 10))
        return -1;
    if (hipSetDevice(dev) != hipSuccess) return -2;
    uint64_t* d = nullptr;
    const size_t bytes = sizeof(uint64_t) * 4 * 4 * (size_t)nwg;  // 4 waves per workgroup
    if (hipMalloc(&d, bytes + sizeof(uint64_t)) != hipSuccess) return -3;
    uint64_t now = 0;
    hipLaunchKernelGGL(realtime_now, dim3(1), dim3(64), 0, 0, d + 4 * 4 * (size_t)nwg);
    if (hipGetLastError() != hipSuccess || hipMemset(d, 0, bytes) != hipSuccess ||
        hipMemcpy(&now, d + 4 * 4 * (size_t)nwg, sizeof now, hipMemcpyDeviceToHost) != hipSuccess) {
        (void)hipFree(d);
        return -4;
    }
    const uint64_t r_start = now + (uint64_t)(delay_s * 1e8), r_end = r_start + (uint64_t)(seconds * 1e8);
    hipLaunchKernelGGL(kFns[kind], dim3(nwg), dim3(256), 0, 0, d, 0x2545f491u, r_start, r_end);
    if (hipGetLastError() != hipSuccess) {
        (void)hipDeviceSynchronize();
        (void)hipFree(d);
        return -5;
    }
    g_slot[dev].out = d;
    g_slot[dev].nwg = nwg;
    return 0;
}

extern "C" int ve_wait(int dev, uint64_t* out, int nwg) {
    if (dev < 0 || dev >= kMaxDevices || !g_slot[dev].out || nwg != g_slot[dev].nwg) return -1;
    if (hipSetDevice(dev) != hipSuccess) return -2;
    uint64_t* d = g_slot[dev].out;
    int rc = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, d, sizeof(uint64_t) * 4 * 4 * (size_t)nwg, hipMemcpyDeviceToHost) != hipSuccess)
        rc = -3;
    (void)hipFree(d);
    g_slot[dev].out = nullptr;
    return rc;
}
