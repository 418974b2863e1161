// Microbenchmark: v_mfma_i32_32x32x32_i8 issue rate on gfx950 (CH independent int32 accumulator
// chains per wave, 1 or 2 waves per SIMD, random operand bytes: the clock the chip holds under
// int8 MFMA load depends on the data). Prints SIMD-cycles per MFMA at the nominal clock and TOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int CH>
__global__ __launch_bounds__(256) void k(int *out, int iters, unsigned seed) {
    v16i acc[CH];
    for (int i = 0; i < CH; ++i)
        for (int r = 0; r < 16; ++r) acc[i][r] = 0;
    unsigned s = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
    v4i a, b;
    for (int r = 0; r < 4; ++r) {
        s = s * 1664525u + 1013904223u; a[r] = (int)s;
        s = s * 1664525u + 1013904223u; b[r] = (int)s;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
    }
    int t = 0;
    for (int i = 0; i < CH; ++i)
        for (int r = 0; r < 16; ++r) t += acc[i][r];
    if (t == 123456789) out[0] = t;
}

template <int CH>
void run(int cus, double clk, int *out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 8192 / CH;
    for (int bpc = 1; bpc <= 2; ++bpc) {
        const int blocks = cus * bpc;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), 0, 0, out, iters, 12345u + rep);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2) {
                const double mfma = blocks * 4.0 * iters * CH;
                const double cyc = ms * 1e-3 * clk * cus * 4.0 / mfma;
                printf("mfma_i32_32x32x32_i8 chains=%d waves/SIMD=%d  %.3f ms  %.2f SIMD-cycles/MFMA @%.0f MHz  %.0f TOP/s\n",
                       CH, bpc, ms, cyc, clk / 1e6, mfma * 65536.0 / (ms * 1e-3) / 1e12);
                fflush(stdout);
            }
        }
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const double clk = p.clockRate * 1e3;
    const int cus = p.multiProcessorCount;
    int *out;
    hipMalloc(&out, 16);
    run<2>(cus, clk, out);
    run<4>(cus, clk, out);
    run<9>(cus, clk, out);
    return 0;
}
