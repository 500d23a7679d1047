// bqp_wave.h — wavefront-level helpers shared by the HIP kernels (gfx950, wave64): intra-wave
// sync, DPP reductions, readlane broadcast, fast reciprocal.  Device code only.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace bqp {

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-wide reductions on DPP lane moves (quad_perm xor1/xor2, row_half_mirror, row_mirror
// inside each 16-lane row, then row_bcast15/31 across rows) + a readlane of lane 63: no LDS
// traffic, result uniform in every lane.  EXEC must be full (all call sites are wave-uniform).
template <int CTRL, int ROWM>
__device__ __forceinline__ double dpp_mov(double old, double v) {
    const int2 o = __builtin_bit_cast(int2, old);
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(o.x, x.x, CTRL, ROWM, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(o.y, x.y, CTRL, ROWM, 0xf, false);
    return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double lane63(double v) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(x.x, 63);
    r.y = __builtin_amdgcn_readlane(x.y, 63);
    return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double wsum(double v) {
    v += dpp_mov<0xB1, 0xf>(0.0, v);
    v += dpp_mov<0x4E, 0xf>(0.0, v);
    v += dpp_mov<0x141, 0xf>(0.0, v);
    v += dpp_mov<0x140, 0xf>(0.0, v);
    v += dpp_mov<0x142, 0xa>(0.0, v);
    v += dpp_mov<0x143, 0xc>(0.0, v);
    return lane63(v);
}
__device__ __forceinline__ double wmax(double v) {
    v = fmax(v, dpp_mov<0xB1, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x4E, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x141, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x140, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x142, 0xa>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x143, 0xc>(-INFINITY, v));
    return lane63(v);
}
__device__ __forceinline__ double wmin(double v) { return -wmax(-v); }
// value of lane `src` broadcast to the wave (scalar register pair): the sequential Riccati
// sweeps pass their NS-vector from stage to stage this way instead of through LDS
__device__ __forceinline__ double rl(double v, int src) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(x.x, src);
    r.y = __builtin_amdgcn_readlane(x.y, src);
    return __builtin_bit_cast(double, r);
}

// fp32 overloads (the structured kernel's fp32 instantiation, bqp_ocp_f32.hip)
template <int CTRL, int ROWM>
__device__ __forceinline__ float dpp_mov(float old, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                  __builtin_bit_cast(int, v), CTRL,
                                                                  ROWM, 0xf, false));
}
__device__ __forceinline__ float lane63(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ float wsum(float v) {
    v += dpp_mov<0xB1, 0xf>(0.0f, v);
    v += dpp_mov<0x4E, 0xf>(0.0f, v);
    v += dpp_mov<0x141, 0xf>(0.0f, v);
    v += dpp_mov<0x140, 0xf>(0.0f, v);
    v += dpp_mov<0x142, 0xa>(0.0f, v);
    v += dpp_mov<0x143, 0xc>(0.0f, v);
    return lane63(v);
}
__device__ __forceinline__ float wmax(float v) {
    v = fmaxf(v, dpp_mov<0xB1, 0xf>(-INFINITY, v));
    v = fmaxf(v, dpp_mov<0x4E, 0xf>(-INFINITY, v));
    v = fmaxf(v, dpp_mov<0x141, 0xf>(-INFINITY, v));
    v = fmaxf(v, dpp_mov<0x140, 0xf>(-INFINITY, v));
    v = fmaxf(v, dpp_mov<0x142, 0xa>(-INFINITY, v));
    v = fmaxf(v, dpp_mov<0x143, 0xc>(-INFINITY, v));
    return lane63(v);
}
__device__ __forceinline__ float wmin(float v) { return -wmax(-v); }
__device__ __forceinline__ float rl(float v, int src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

}  // namespace bqp
