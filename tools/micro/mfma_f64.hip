// Microbenchmark: v_mfma_f64_16x16x4_f64 issue rate on gfx950 (8 independent accumulator
// chains per wave, 1..4 waves per SIMD). Prints SIMD-cycles per MFMA and TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(256) void k(double *out, int iters, double a) {
    d4 acc[CH];
    for (int i = 0; i < CH; ++i) acc[i] = d4{0.0, 0.0, 0.0, (double)threadIdx.x};
    double x = a + threadIdx.x * 1e-9, y = a - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < CH; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.678) out[0] = s;
}

template <int CH>
void run(int cus, double clk, double *out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 16384 / CH;
    for (int bpc = 1; bpc <= 4; bpc *= 2) {
        const int blocks = cus * bpc;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 1) {
                const double mfma = blocks * 4.0 * iters * CH;
                const double cyc = ms * 1e-3 * clk * cus * 4.0 / mfma;
                printf("mfma_f64_16x16x4 chains=%d waves/SIMD=%d  %.3f ms  %.2f SIMD-cycles/MFMA @%.0f MHz  %.1f TFLOP/s\n",
                       CH, bpc, ms, cyc, clk / 1e6, mfma * 2048.0 / (ms * 1e-3) / 1e12);
            }
        }
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const double clk = p.clockRate * 1e3;
    const int cus = p.multiProcessorCount;
    double *out;
    hipMalloc(&out, 16);
    run<1>(cus, clk, out);
    run<2>(cus, clk, out);
    run<4>(cus, clk, out);
    run<8>(cus, clk, out);
    return 0;
}
