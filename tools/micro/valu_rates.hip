// Microbenchmark: wave64 VALU issue rates on gfx950 (fp64 FMA, fp64 mul+cmp, fp32 FMA,
// int ops). Many waves per SIMD, 8 independent chains per lane. Prints per-instruction
// cycles per SIMD assuming the clock reported by hipDeviceProp (clockRate).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(256) void k(double *out, int iters, double a, double b) {
    double v[8];
    float f[8];
    unsigned u[8];
    for (int i = 0; i < 8; ++i) { v[i] = threadIdx.x * 1e-3 + i; f[i] = (float)v[i]; u[i] = threadIdx.x + i; }
    unsigned cnt = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (KIND == 0) v[i] = fma(v[i], a, b);
            if (KIND == 1) f[i] = fmaf(f[i], (float)a, (float)b);
            if (KIND == 2) u[i] = (u[i] ^ (u[i] >> 3)) + 0x9e37u;     // 2 int ops
            if (KIND == 3) { v[i] = v[i] * a; cnt += v[i] > b; }        // mul + cmp + cndmask/add
        }
    }
    double s = 0;
    for (int i = 0; i < 8; ++i) s += v[i] + f[i] + u[i];
    if (s == 12345.678) out[0] = s + cnt;
    if (cnt == 0xffffffffu) out[1] = 1;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const double clk = p.clockRate * 1e3;   // Hz
    const int cus = p.multiProcessorCount;
    double *out;
    hipMalloc(&out, 16);
    const int iters = 4096, blocks = cus * 8;   // 8 blocks x 4 waves per CU = 8 waves/SIMD
    const char *names[] = {"v_fma_f64", "v_fma_f32", "int xor/shr/add (per 3 ops)", "v_mul_f64 + v_cmp_f64 + add"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int kind = 0; kind < 4; ++kind) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
            if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
            if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
            if (kind == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 1) {
                const double waves = blocks * 4.0, inst = waves * iters * 8.0;   // per-chain steps
                const double simds = cus * 4.0;
                const double cyc = ms * 1e-3 * clk * simds / inst;
                printf("%-34s %.3f ms  %.2f SIMD-cycles per wave64 step (clk %.0f MHz, %d CUs)\n", names[kind], ms, cyc,
                       clk / 1e6, cus);
            }
        }
    }
    return 0;
}
