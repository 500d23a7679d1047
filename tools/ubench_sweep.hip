// ubench_sweep.hip — diagnostic: cycles per step of candidate Riccati-sweep step forms on gfx950
// (p_k = Phi' p_{k+1} + q, 5-vector, lane i < 5 owns entry i).  Not part of the product.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define STEPS 400
#define NS 5

__device__ __forceinline__ double rl(double v, int src) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(x.x, src);
    r.y = __builtin_amdgcn_readlane(x.y, src);
    return __builtin_bit_cast(double, r);
}
// SGPR -> VGPR copy the compiler cannot fold into the consumer
__device__ __forceinline__ double to_v(double s) {
    double v;
    asm volatile("v_mov_b64 %0, %1" : "=v"(v) : "s"(s));
    return v;
}
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(64) sw(int mode, const double* phi_g, double* out,
                                          unsigned long long* cyc) {
    __shared__ double lds[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) lds[i] = phi_g[i & 255];
    __syncthreads();
    const int li = lane < NS ? lane : NS - 1;
    double p[NS];
#pragma unroll
    for (int c = 0; c < NS; ++c) p[c] = 0.1 * (c + 1);
    double pv = 0.1 * (li + 1);
    double ph[NS];
#pragma unroll
    for (int c = 0; c < NS; ++c) ph[c] = lds[c * NS + li] * 0.2;
    const double q = 1e-3 * lane;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {            // current: FMA chain over readlane'd p (SGPR operands)
        for (int k = 0; k < STEPS; ++k) {
            double acc = q;
#pragma unroll
            for (int c = 0; c < NS; ++c) acc += ph[c] * p[c];
#pragma unroll
            for (int c = 0; c < NS; ++c) p[c] = rl(acc, c);
        }
        pv = p[0];
    } else if (mode == 1) {     // independent products (SGPR) + VGPR tree
        for (int k = 0; k < STEPS; ++k) {
            double m[NS];
#pragma unroll
            for (int c = 0; c < NS; ++c) m[c] = ph[c] * p[c];
            const double acc = ((m[0] + m[1]) + (m[2] + m[3])) + (m[4] + q);
#pragma unroll
            for (int c = 0; c < NS; ++c) p[c] = rl(acc, c);
        }
        pv = p[0];
    } else if (mode == 2) {     // readlane + forced VGPR copy, FMA chain on VGPRs
        for (int k = 0; k < STEPS; ++k) {
            double acc = q;
#pragma unroll
            for (int c = 0; c < NS; ++c) acc = __builtin_fma(ph[c], p[c], acc);
#pragma unroll
            for (int c = 0; c < NS; ++c) p[c] = to_v(rl(acc, c));
        }
        pv = p[0];
    } else if (mode == 3) {     // readlane + forced VGPR copy + tree
        for (int k = 0; k < STEPS; ++k) {
            double m[NS];
#pragma unroll
            for (int c = 0; c < NS; ++c) m[c] = ph[c] * p[c];
            const double acc = ((m[0] + m[1]) + (m[2] + m[3])) + (m[4] + q);
#pragma unroll
            for (int c = 0; c < NS; ++c) p[c] = to_v(rl(acc, c));
        }
        pv = p[0];
    } else if (mode == 4) {     // LDS broadcast: lanes < NS store, wave sync, all read
        for (int k = 0; k < STEPS; ++k) {
            double m[NS];
#pragma unroll
            for (int c = 0; c < NS; ++c) m[c] = ph[c] * p[c];
            const double acc = ((m[0] + m[1]) + (m[2] + m[3])) + (m[4] + q);
            double* slot = lds + 2048 + (k & 63) * 8;
            if (lane < NS) slot[lane] = acc;
            wsync();
#pragma unroll
            for (int c = 0; c < NS; ++c) p[c] = slot[c];
        }
        pv = p[0];
    } else if (mode == 5) {     // DPP-free: every lane computes the whole vector (25 FMAs, VGPR)
        double pp[NS];
#pragma unroll
        for (int c = 0; c < NS; ++c) pp[c] = p[c] + lane * 1e-9;
        double PH[NS][NS];
#pragma unroll
        for (int i = 0; i < NS; ++i)
#pragma unroll
            for (int c = 0; c < NS; ++c) PH[i][c] = lds[c * NS + i] * 0.2;
        for (int k = 0; k < STEPS; ++k) {
            double nw[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                double m0 = PH[i][0] * pp[0], m1 = PH[i][1] * pp[1];
                double m2 = PH[i][2] * pp[2], m3 = PH[i][3] * pp[3];
                nw[i] = ((m0 + m1) + (m2 + m3)) + __builtin_fma(PH[i][4], pp[4], q);
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) pp[i] = nw[i];
        }
        pv = pp[0];
    }
    __builtin_amdgcn_s_waitcnt(0);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = pv;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    double *phi, *out;
    unsigned long long* cyc;
    (void)hipMalloc(&phi, 256 * sizeof(double));
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&cyc, sizeof(unsigned long long));
    double h[256];
    for (int i = 0; i < 256; ++i) h[i] = 0.3 + 0.001 * i;
    (void)hipMemcpy(phi, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[] = {"fma chain, SGPR p (current)", "SGPR products + VGPR tree",
                           "fma chain, VGPR copies", "VGPR copies + tree", "LDS broadcast + tree",
                           "all lanes full 5x5 (no exchange)"};
    for (int mode = 0; mode < 6; ++mode) {
        unsigned long long c = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(sw, dim3(1), dim3(64), 0, 0, mode, phi, out, cyc);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        }
        printf("%-36s %8.1f cyc/step\n", names[mode], (double)c / STEPS);
    }
    return 0;
}
