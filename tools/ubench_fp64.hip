// ubench_fp64.hip — diagnostic microbenchmarks of the gfx950 latencies that bound the
// structured kernel's critical path (not part of the product).  One 512-thread workgroup;
// only wave 0 (and wave 4, which shares its SIMD, when `pair` is set) run the test.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_fp64.hip -o build/ubench && ./build/ubench
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REPS 512

__device__ __forceinline__ double rl(double v, int src) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(x.x, src);
    r.y = __builtin_amdgcn_readlane(x.y, src);
    return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double dppx1(double v) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(0, x.x, 0xB1, 0xf, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(0, x.y, 0xB1, 0xf, 0xf, false);
    return __builtin_bit_cast(double, r);
}

__global__ void __launch_bounds__(512) ub(int mode, int pair, double a, double b, double* out,
                                           unsigned long long* cyc) {
    __shared__ double lds[1024];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 1024; i += 512) lds[i] = 1.0 + 1e-3 * i;
    __syncthreads();
    if (!(w == 0 || (pair && w == 4))) return;
    double x0 = 1.0 + lane * 1e-6, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,
           x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    int idx = lane;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (mode) {
        case 0:   // dependent fp64 FMA chain
            for (int i = 0; i < REPS; ++i) x0 = __builtin_fma(x0, a, b);
            break;
        case 1:   // 8 independent fp64 FMA chains (throughput of one wave)
            for (int i = 0; i < REPS; ++i) {
                x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b);
                x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
                x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b);
                x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
            }
            break;
        case 2:   // dependent v_rcp_f64 + 2 Newton steps (frcp of the kernel)
            for (int i = 0; i < REPS; ++i) {
                double r = __builtin_amdgcn_rcp(x0);
                double e = __builtin_fma(-x0, r, 1.0);
                r = __builtin_fma(r, e, r);
                e = __builtin_fma(-x0, r, 1.0);
                x0 = __builtin_fma(r, e, r) + b;
            }
            break;
        case 3:   // readlane broadcast chain: x = fma(readlane(x, k), a, b)
            for (int i = 0; i < REPS; ++i) x0 = __builtin_fma(rl(x0, i & 7), a, b);
            break;
        case 4:   // DPP exchange chain
            for (int i = 0; i < REPS; ++i) x0 = x0 + dppx1(x0) * a;
            break;
        case 5:   // LDS store by one lane -> wave barrier -> broadcast read, dependent
            for (int i = 0; i < REPS; ++i) {
                if (lane == (i & 15)) lds[512 + (i & 255)] = x0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                x0 = __builtin_fma(lds[512 + (i & 255)], a, b);
            }
            break;
        case 6:   // dependent ds_read_b64 (address from data)
            for (int i = 0; i < REPS; ++i) {
                const double v = lds[idx];
                idx = ((int)v + lane + i) & 511;
                x0 += v;
            }
            break;
        case 7:   // 4 independent fp64 FMA chains
            for (int i = 0; i < REPS; ++i) {
                x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b);
                x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
            }
            break;
        case 8:   // 8 independent fp32 FMA chains (reference for the issue cost)
        {
            float f0 = x0, f1 = x1, f2 = x2, f3 = x3, f4 = x4, f5 = x5, f6 = x6, f7 = x7;
            const float fa = a, fb = b;
            for (int i = 0; i < REPS; ++i) {
                f0 = __builtin_fmaf(f0, fa, fb); f1 = __builtin_fmaf(f1, fa, fb);
                f2 = __builtin_fmaf(f2, fa, fb); f3 = __builtin_fmaf(f3, fa, fb);
                f4 = __builtin_fmaf(f4, fa, fb); f5 = __builtin_fmaf(f5, fa, fb);
                f6 = __builtin_fmaf(f6, fa, fb); f7 = __builtin_fmaf(f7, fa, fb);
            }
            x0 = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
            break;
        }
        case 9:   // dependent fp64 mul+add pair (v_mul_f64 then v_add_f64)
            for (int i = 0; i < REPS; ++i) x0 = x0 * a + b;
            break;
        case 10: {  // dependent fp64 FMA chain, VGPR-only operands (lane-varying a, b)
            const double va = a + lane * 1e-12, vb = b + lane * 1e-15;
            for (int i = 0; i < REPS; ++i) x0 = __builtin_fma(x0, va, vb);
            break;
        }
        case 11: {  // dependent fp64 add chain, VGPR operand
            const double vb = b + lane * 1e-15;
            for (int i = 0; i < REPS; ++i) x0 = x0 + vb;
            break;
        }
        case 12: {  // dependent fp32 FMA chain, VGPR operands
            float f = x0; const float fa = a + lane * 1e-9f, fb = b;
            for (int i = 0; i < REPS; ++i) f = __builtin_fmaf(f, fa, fb);
            x0 = f;
            break;
        }
        case 13: {  // two interleaved dependent fp64 FMA chains, VGPR operands
            const double va = a + lane * 1e-12, vb = b + lane * 1e-15;
            for (int i = 0; i < REPS; ++i) { x0 = __builtin_fma(x0, va, vb); x1 = __builtin_fma(x1, va, vb); }
            break;
        }
        case 14: {  // dependent fp64 mul chain VGPR
            const double va = a + lane * 1e-12;
            for (int i = 0; i < REPS; ++i) x0 = x0 * va;
            break;
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if (lane == 0) cyc[w] = t1 - t0;
}

int main() {
    double* out;
    unsigned long long* cyc;
    hipMalloc(&out, 512 * sizeof(double));
    hipMalloc(&cyc, 8 * sizeof(unsigned long long));
    const char* names[] = {"dep fma f64", "8 indep fma f64 (per instr)", "frcp chain (rcp+4 fma)",
                           "readlane->fma chain", "dpp->fma chain", "lds st/sync/ld chain",
                           "dep ds_read_b64", "4 indep fma f64 (per instr)",
                           "8 indep fma f32 (per instr)", "dep mul+add f64 (pair)",
                           "dep fma f64 VGPR-only", "dep add f64 VGPR", "dep fma f32 VGPR",
                           "2 interleaved dep fma f64 (per instr)", "dep mul f64 VGPR"};
    const double per[] = {1, 8, 1, 1, 1, 1, 1, 4, 8, 1, 1, 1, 1, 2, 1};
    for (int pair = 0; pair < 2; ++pair)
        for (int mode = 0; mode < 15; ++mode) {
            unsigned long long h[8] = {0};
            for (int rep = 0; rep < 3; ++rep) {
                hipMemset(cyc, 0, 8 * sizeof(unsigned long long));
                hipLaunchKernelGGL(ub, dim3(1), dim3(512), 0, 0, mode, pair, 0.999999, 1e-7, out, cyc);
                hipDeviceSynchronize();
                hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
            }
            printf("%s %-32s %8.2f cyc/op (wave0 %llu, wave4 %llu)\n", pair ? "2 waves/SIMD" : "1 wave     ",
                   names[mode], (double)h[0] / (REPS * per[mode]), h[0], h[4]);
        }
    return 0;
}
