// wave_ops.hpp -- 64-lane wavefront primitives for the one-QP-per-wavefront kernels (gfx950).
//
// Every kernel in this library runs one problem instance per 64-lane wavefront (one wave per
// workgroup), so all control flow inside an instance is wave-uniform and these helpers can
// assume a full, converged wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpcqp {

constexpr int kWave = 64;

__device__ __forceinline__ int lane() { return (int)__lane_id(); }

// Broadcast lane `src` (wave-uniform index) of a double to the whole wave (v_readlane x2).
__device__ __forceinline__ double readlane(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int readlane(int v, int src) {
    return __builtin_amdgcn_readlane(v, src);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
    return v;
}
// lexicographic (value, index) minimum; lanes with nothing to offer pass (+inf, INT_MAX)
__device__ __forceinline__ void wave_argmin(double &v, int &idx) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, kWave);
        const int oi = __shfl_xor(idx, o, kWave);
        if (ov < v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
}
// (value, index) maximum with the lowest index winning ties (Eigen maxCoeff semantics)
__device__ __forceinline__ void wave_argmax(double &v, int &idx) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, kWave);
        const int oi = __shfl_xor(idx, o, kWave);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
}

// Ordering point between phases of a single-wave workgroup.  One wave issues its LDS
// instructions in program order and the LDS executes them in order, so a store by one lane
// is seen by a later load of another lane without any wait; only the compiler must not move
// LDS accesses across this point (wavefront-scope fences emit no instruction).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Code-motion fence for unrolled straight-line phases: no memory access moves across it at
// the IR level (empty asm with a memory clobber) nor in the machine scheduler.
__device__ __forceinline__ void step_fence() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// Materialise v in a VGPR at this point: arithmetic producing v cannot sink past it.
__device__ __forceinline__ void pin(double &v) { asm volatile("" : "+v"(v)); }

// Diagnostic phase stamps (built only with -DMPCQP_STAMPS, lib/libmpcqp_stamps.so): cycles
// (s_memtime) since the previous stamp are added to slot k of a global array.  The real
// library compiles these to nothing.
#ifdef MPCQP_STAMPS
#define MPCQP_STAMP(ptr, k, t)                                                  \
    do {                                                                        \
        if (ptr) {                                                              \
            const unsigned long long now_ = __builtin_amdgcn_s_memtime();      \
            if (::mpcqp::lane() == 0) atomicAdd(&(ptr)[(k)], now_ - (t));      \
            (t) = now_;                                                         \
        }                                                                       \
    } while (0)
#define MPCQP_STAMP_INIT(t) unsigned long long t = __builtin_amdgcn_s_memtime()
#else
#define MPCQP_STAMP(ptr, k, t) ((void)0)
#define MPCQP_STAMP_INIT(t) ((void)0)
#endif

}  // namespace mpcqp
