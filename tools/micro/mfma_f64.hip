// Microbenchmark: v_mfma_f64_16x16x4_f64 issue rate on gfx950 (8 independent accumulator
// chains per wave, 1..4 waves per SIMD). Prints SIMD-cycles per MFMA and TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k(double *out, int iters, double a) {
    d4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = d4{0.0, 0.0, 0.0, (double)threadIdx.x};
    double x = a + threadIdx.x * 1e-9, y = a - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.678) out[0] = s;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const double clk = p.clockRate * 1e3;
    const int cus = p.multiProcessorCount;
    double *out;
    hipMalloc(&out, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2048;
    for (int bpc = 1; bpc <= 4; bpc *= 2) {
        const int blocks = cus * bpc;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 1) {
                const double mfma = blocks * 4.0 * iters * 8.0;
                const double cyc = ms * 1e-3 * clk * cus * 4.0 / mfma;
                printf("mfma_f64_16x16x4 waves/SIMD=%d  %.3f ms  %.2f SIMD-cycles/MFMA  %.1f TFLOP/s (clk %.0f MHz)\n", bpc,
                       ms, cyc, mfma * 2048.0 / (ms * 1e-3) / 1e12, clk / 1e6);
            }
        }
    }
    return 0;
}
