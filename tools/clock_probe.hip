// clock_probe.hip -- the engine clock a kernel runs at, measured from inside the GPU while it runs.
//
// MI355X lowers its clock under load, and a profiled run clocks lower than an un-profiled one
// (MI355X_MICROARCH.md "DVFS give-back" items 2 and 6), so neither rocprofv3's GRBM_GUI_ACTIVE
// pass nor amd-smi's reading is the clock of the bench's own search.  This probe is a separate
// kernel on its own stream: a few one-wave workgroups that sleep through the search and read the
// shader-clock counter (s_memtime) and the 100 MHz constant counter (s_memrealtime) at both ends
// of a window that lies inside the search.  Clock = d(memtime) / d(memrealtime) x 100 MHz, per
// workgroup, with the XCD it ran on (HW_REG_XCC_ID).  The product kernel carries no stamp.
//
// The probe waves only sleep and read counters (~8 VGPRs each), so at most they take one wave
// slot on a few SIMDs from the search.  Results go to a buffer of their own by vector stores.
//
// C-ABI (build/libclockprobe.so, loaded by bench.py with ctypes; measurement only):
//   cp_start(dev, delay_s, window_s, nwg)  launch nwg probe workgroups on device dev, return at once
//   cp_read(dev, out, nwg)                 wait for them; out[4*i..4*i+3] = {xcc, cycles,
//                                          100 MHz ticks, ticks from the workgroup's start to
//                                          its window}
// One probe at a time per device; probes on different devices may run at once, each started and
// read from its own host thread (bench.py's in-process N-GPU lines read every device's clock
// during concurrent searches).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr uint64_t kRealtimeHz = 100000000ull;  // s_memrealtime: constant 100 MHz
// s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): id 20, offset 0, size 4 -> 20 | (3 << 11)
constexpr int kXccIdReg = 20 | (3 << 11);

__global__ void clock_probe(uint64_t* __restrict__ out, uint64_t delay_ticks, uint64_t window_ticks) {
    const uint64_t r_start = __builtin_amdgcn_s_memrealtime();
    uint64_t r = r_start;
    while (r - r_start < delay_ticks) {  // let the search reach its steady clock first
        __builtin_amdgcn_s_sleep(127);
        r = __builtin_amdgcn_s_memrealtime();
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    r = r0;
    while (r - r0 < window_ticks) {
        __builtin_amdgcn_s_sleep(127);
        r = __builtin_amdgcn_s_memrealtime();
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(kXccIdReg);
    if (threadIdx.x < 4) {
        const uint64_t v[4] = {xcc, t1 - t0, r1 - r0, r0 - r_start};
        out[4 * (uint64_t)blockIdx.x + threadIdx.x] = v[threadIdx.x];
    }
}

constexpr int kMaxDevices = 64;
struct Slot {
    hipStream_t stream = nullptr;  // created on the slot's device
    uint64_t* out = nullptr;       // non-null while a probe is outstanding
    int nwg = 0;
};
Slot g_slot[kMaxDevices];  // slot d is touched only by the thread that probes device d

}  // namespace

extern "C" int cp_start(int dev, double delay_s, double window_s, int nwg) {
    if (dev < 0 || dev >= kMaxDevices) return -1;
    Slot& s = g_slot[dev];
    if (nwg < 1 || nwg > 4096 || delay_s < 0 || window_s <= 0 || s.out) return -1;
    if (hipSetDevice(dev) != hipSuccess) return -2;
    if (!s.stream && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return -3;
    if (hipMalloc(&s.out, sizeof(uint64_t) * 4 * nwg) != hipSuccess) {
        s.out = nullptr;
        return -4;
    }
    if (hipMemsetAsync(s.out, 0, sizeof(uint64_t) * 4 * nwg, s.stream) != hipSuccess) {
        (void)hipFree(s.out);
        s.out = nullptr;
        return -5;
    }
    s.nwg = nwg;
    hipLaunchKernelGGL(clock_probe, dim3(nwg), dim3(64), 0, s.stream, s.out,
                       (uint64_t)(delay_s * kRealtimeHz), (uint64_t)(window_s * kRealtimeHz));
    if (hipGetLastError() != hipSuccess) {  // nothing runs: free the buffer so a later start works
        (void)hipStreamSynchronize(s.stream);
        (void)hipFree(s.out);
        s.out = nullptr;
        return -6;
    }
    return 0;
}

extern "C" int cp_read(int dev, uint64_t* out, int nwg) {
    if (dev < 0 || dev >= kMaxDevices) return -1;
    Slot& s = g_slot[dev];
    if (!s.out || nwg != s.nwg) return -1;
    if (hipSetDevice(dev) != hipSuccess) return -2;
    int rc = 0;
    if (hipStreamSynchronize(s.stream) != hipSuccess ||
        hipMemcpy(out, s.out, sizeof(uint64_t) * 4 * nwg, hipMemcpyDeviceToHost) != hipSuccess)
        rc = -3;
    (void)hipFree(s.out);
    s.out = nullptr;
    return rc;
}
