// Device check of the transposed multi-value wave sum (bqp_wave.h wsum_t): lane l must hold
// the wave total of value (l & 31).  Built by learning-based-mpc_amd/Makefile (build/wsum_t_check),
// run by tests/test_gpu_wave.py.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include "bqp_wave.h"
using namespace bqp;
template <int K>
__global__ void k(const double* in, double* out) {
    const int lane = threadIdx.x;
    double v[K];
    for (int c = 0; c < K; ++c) v[c] = in[lane * K + c];
    out[lane] = wsum_t(v, lane);
}
template <int K>
int run() {
    double h[64 * K], o[64], *di, *dout;
    for (int i = 0; i < 64 * K; ++i) h[i] = sin(1.0 + i * 0.37) * (1 + (i % 7));
    hipMalloc(&di, sizeof h); hipMalloc(&dout, sizeof o);
    hipMemcpy(di, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k<K>, dim3(1), dim3(64), 0, 0, di, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    double err = 0;
    for (int l = 0; l < 64; ++l) {
        const int id = l & 31;
        double s = 0;
        if (id < K) for (int j = 0; j < 64; ++j) s += h[j * K + id];
        err = fmax(err, fabs(s - o[l]));
    }
    printf("K=%d max err %.3e\n", K, err);
    return err < 1e-12 ? 0 : 1;
}
int main() { return run<28>() | run<13>() | run<6>() | run<2>(); }
