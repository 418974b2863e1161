// Microbenchmark: fp64 VALU issue rate vs waves per SIMD on gfx950 (what bounds the CI-test
// kernels). W waves per SIMD = W blocks of 256 threads per CU. Each lane runs NCH independent
// chains of v_fma_f64 (KIND 0) or of 32-bit integer ops (KIND 2). Prints SIMD-cycles per
// wave64 instruction using the shader clock measured in-kernel (s_memtime against the
// 100 MHz s_memrealtime), so DVFS does not distort the cycle counts.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND, int NCH>
__global__ __launch_bounds__(256) void k(double *out, unsigned long long *clk, int iters, double a, double b) {
    double v[NCH];
    unsigned u[NCH];
    for (int i = 0; i < NCH; ++i) { v[i] = threadIdx.x * 1e-3 + i; u[i] = threadIdx.x + i; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            if (KIND == 0) v[i] = fma(v[i], a, b);
            if (KIND == 2) u[i] = (u[i] ^ (u[i] >> 3)) + 0x9e37u;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
    for (int i = 0; i < NCH; ++i) s += v[i] + u[i];
    if (s == 12345.678) out[0] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int KIND, int NCH>
void run(int W, int cus) {
    double *out;
    unsigned long long *clk, hc[2];
    (void)hipMalloc(&out, 16);
    (void)hipMalloc(&clk, 16);
    const int iters = 16384, blocks = cus * W;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k<KIND, NCH>), dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0000001, 1e-9);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    (void)hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)hc[0] / ((double)hc[1] / 100e6) / 1e9;   // memrealtime is 100 MHz
    const double instr = (double)W * iters * NCH * (KIND == 2 ? 3.0 : 1.0);
    printf("  kind %d chains %d: %.2f cyc/instr (in-kernel clock %.2f GHz, wall %.3f ms, %.2f cyc at wall)\n", KIND,
           NCH, (double)hc[0] / instr, ghz, ms, ms * 1e-3 * ghz * 1e9 / instr);
    (void)hipFree(out);
    (void)hipFree(clk);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("%d CUs, max clock %.0f MHz\n", cus, p.clockRate / 1e3);
    for (int W : {1, 2, 3, 4, 6, 8}) {
        printf("waves/SIMD %d\n", W);
        run<0, 8>(W, cus);
        run<0, 4>(W, cus);
        run<2, 8>(W, cus);
    }
    return 0;
}
