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

// ---- transposed multi-value sums: K <= 32 per-lane partials reduced over the wave at once ----
// Each exchange step halves the number of values a lane carries: of a pair (a, b) a lane keeps a
// or b by one bit of its lane id and adds the partner lane's other one (quad_perm xor1, xor2,
// row_ror 4, row_ror 8 inside 16-lane rows; then the gfx950 row swaps v_permlane16_swap /
// v_permlane32_swap across rows).  K values cost ~K pair steps instead of 6 K DPP steps.
// Afterwards lane l holds the wave total of value (l & 31) (0 for ids >= K).
__device__ __forceinline__ void pl16_swap(double& a, double& b) {
    const int2 A = __builtin_bit_cast(int2, a), B = __builtin_bit_cast(int2, b);
    const auto x = __builtin_amdgcn_permlane16_swap((unsigned)A.x, (unsigned)B.x, false, false);
    const auto y = __builtin_amdgcn_permlane16_swap((unsigned)A.y, (unsigned)B.y, false, false);
    a = __builtin_bit_cast(double, make_int2((int)x[0], (int)y[0]));
    b = __builtin_bit_cast(double, make_int2((int)x[1], (int)y[1]));
}
__device__ __forceinline__ void pl32_swap(double& a, double& b) {
    const int2 A = __builtin_bit_cast(int2, a), B = __builtin_bit_cast(int2, b);
    const auto x = __builtin_amdgcn_permlane32_swap((unsigned)A.x, (unsigned)B.x, false, false);
    const auto y = __builtin_amdgcn_permlane32_swap((unsigned)A.y, (unsigned)B.y, false, false);
    a = __builtin_bit_cast(double, make_int2((int)x[0], (int)y[0]));
    b = __builtin_bit_cast(double, make_int2((int)x[1], (int)y[1]));
}
__device__ __forceinline__ void pl16_swap(float& a, float& b) {
    const auto x = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a),
                                                    __builtin_bit_cast(unsigned, b), false, false);
    a = __builtin_bit_cast(float, (unsigned)x[0]);
    b = __builtin_bit_cast(float, (unsigned)x[1]);
}
__device__ __forceinline__ void pl32_swap(float& a, float& b) {
    const auto x = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a),
                                                    __builtin_bit_cast(unsigned, b), false, false);
    a = __builtin_bit_cast(float, (unsigned)x[0]);
    b = __builtin_bit_cast(float, (unsigned)x[1]);
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

// lane C's value in every lane of its 16-lane row (gfx950 DPP row_newbcast: one v_mov_b64_dpp
// / v_mov_b32_dpp, the value stays in vector registers); rbc_all fills p[c] = lane c's v for
// c < NC (NC <= 16), the sweep broadcast without a scalar round trip
template <int C>
__device__ __forceinline__ double rbc(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + C, 0xf, 0xf, false);
}
template <int C>
__device__ __forceinline__ float rbc(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                 0x150 + C, 0xf, 0xf, false));
}
// the value of 16-lane row Q (lane 16 Q + l%16) in lane l of every row: v_permlane16_swap of a
// register with itself gives the even / odd row pairs, v_permlane32_swap the halves - VALU only
// (the ds_bpermute form took an LDS round trip)
template <int Q>
__device__ __forceinline__ double xrow_bcast(double v) {
    double a = v, b = v;
    pl16_swap(a, b);                 // a: rows (0, 0, 2, 2), b: rows (1, 1, 3, 3)
    double c = (Q & 1) ? b : a, d = c;
    pl32_swap(c, d);                 // c: rows (q, q, q, q) of the lower pair, d: of the upper pair
    return (Q >> 1) ? d : c;
}

template <int C, int NC, typename T>
__device__ __forceinline__ void rbc_all(T v, T (&p)[NC]) {
    p[C] = rbc<C>(v);
    if constexpr (C + 1 < NC) rbc_all<C + 1, NC>(v, p);
}

template <int CTRL, typename T, int KI, int KO>
__device__ __forceinline__ void tsum_step(const T (&in)[KI], T (&out)[KO], bool hi) {
#pragma unroll
    for (int p = 0; p < KO; ++p) {
        const T a = in[2 * p];
        const T b = (2 * p + 1 < KI) ? in[2 * p + 1] : T(0);
        const T keep = hi ? b : a;
        const T send = hi ? a : b;
        out[p] = keep + dpp_mov<CTRL, 0xf>(T(0), send);
    }
}
template <typename T, int K>
__device__ __forceinline__ T wsum_t(const T (&v)[K], int lane) {
    static_assert(K >= 2 && K <= 32, "wsum_t: 2..32 values");
    constexpr int K1 = (K + 1) / 2, K2 = (K1 + 1) / 2, K3 = (K2 + 1) / 2, K4 = (K3 + 1) / 2;
    T w1[K1], w2[K2], w3[K3], w4[K4];
    tsum_step<0xB1>(v, w1, (lane & 1) != 0);     // quad_perm [1,0,3,2]
    tsum_step<0x4E>(w1, w2, (lane & 2) != 0);    // quad_perm [2,3,0,1]
    tsum_step<0x124>(w2, w3, (lane & 4) != 0);   // row_ror:4
    tsum_step<0x128>(w3, w4, (lane & 8) != 0);   // row_ror:8
    T a = w4[0], b = T(0);
    if constexpr (K4 > 1) b = w4[K4 - 1];
    pl16_swap(a, b);                             // even rows: value a over rows {0,1} / {2,3}
    T c = a + b, d = c;
    pl32_swap(c, d);                             // halves {0,1} + {2,3}
    return c + d;
}

}  // namespace bqp
