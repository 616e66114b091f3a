// Host-side helpers shared by the C-ABI entry points: per-device one-time work and device
// properties. A process may drive several GPUs through the C-ABI (one device per thread, or a
// loop over devices), so nothing here is a per-process flag: kernel attributes are set once per
// device, the CU count is cached per device, and both are safe to call from several threads.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

namespace evxh {

inline int cur_device() {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess ? d : -1;
}

// Runs f() unless it already ran for the current device (devices 0..63; beyond, every call runs
// it). Two threads may both run it the first time: f must be idempotent (attribute setters are).
template <class F>
inline void once_per_device(std::atomic<uint64_t>& done, F&& f) {
    const int d = cur_device();
    const uint64_t bit = (d >= 0 && d < 64) ? (1ull << d) : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return;
    f();
    if (bit) done.fetch_or(bit, std::memory_order_acq_rel);
}

// Raises a kernel's dynamic-LDS limit on the current device, once per device.
inline void max_lds_once(std::atomic<uint64_t>& done, const void* const* kernels, int n, int bytes) {
    once_per_device(done, [&] {
        for (int i = 0; i < n; i++) (void)hipFuncSetAttribute(kernels[i], hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    });
}

// Compute units of the current device (cached per device; 256 if the query fails).
inline int cu_count() {
    static std::atomic<int> ncu[64];
    const int d = cur_device();
    int n = 0;
    if (d >= 0 && d < 64 && (n = ncu[d].load(std::memory_order_relaxed)) > 0) return n;
    if (d < 0 || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0) n = 256;
    if (d >= 0 && d < 64) ncu[d].store(n, std::memory_order_relaxed);
    return n;
}

}  // namespace evxh
