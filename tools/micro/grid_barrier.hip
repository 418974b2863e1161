// Cost of a software grid barrier on MI355X (the fused level barrier's k_level_end question):
// one launch of B persistent blocks x T threads running K barriers, timed with events, against
// K + 1 back-to-back empty launches (the dependent-kernel alternative). Variants:
//   mode 0: leader-only agent release + relaxed polling + one acquire (k_level_end's grid_sync)
//   mode 1: every thread fences (agent release + acquire) and the leader polls with acquire loads
// Each block also writes and, after the barrier, reads one word per thread of a buffer written
// by another block, so the barrier carries data as in the fused kernel (checked: errors printed).
// usage: grid_barrier [blocks=256] [threads=256] [barriers=8]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

struct Bar {
    unsigned count, gen, abort, pad;
};

template <int MODE>
__device__ void gsync(Bar *g, unsigned nblk) {
    if (MODE == 1) __threadfence();
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned gen = __hip_atomic_load(&g->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned arrived = __hip_atomic_fetch_add(&g->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nblk - 1) {
            (void)__hip_atomic_exchange(&g->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&g->gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned spins = 0;
            while ((MODE == 1 ? __hip_atomic_load(&g->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                              : __hip_atomic_load(&g->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == gen) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > (1u << 22)) {
                    __hip_atomic_store(&g->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                if (__hip_atomic_load(&g->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

template <int MODE>
__global__ void k_barriers(Bar *g, int K, unsigned *buf, unsigned *err) {
    const unsigned nblk = gridDim.x, blk = blockIdx.x, T = blockDim.x;
    for (int k = 0; k < K; ++k) {
        buf[(size_t)blk * T + threadIdx.x] = (unsigned)k * 1000003u + blk;
        gsync<MODE>(g, nblk);
        const unsigned src = (blk + 1 + (unsigned)k) % nblk;     // another block's word
        const unsigned v = buf[(size_t)src * T + threadIdx.x];
        if (v != (unsigned)k * 1000003u + src) atomicAdd(err, 1u);
        gsync<MODE>(g, nblk);
    }
}

__global__ void k_empty(unsigned *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 0xdeadbeefu) p[1] = 1;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 256, T = argc > 2 ? atoi(argv[2]) : 256, K = argc > 3 ? atoi(argv[3]) : 8;
    Bar *g;
    unsigned *buf, *err;
    (void)hipMalloc(&g, sizeof(Bar));
    (void)hipMemset(g, 0, sizeof(Bar));
    (void)hipMalloc(&buf, sizeof(unsigned) * (size_t)B * T);
    (void)hipMalloc(&err, sizeof(unsigned));
    (void)hipMemset(err, 0, sizeof(unsigned));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int mode = 0; mode < 2; ++mode) {
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            (void)hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(k_barriers<0>, dim3(B), dim3(T), 0, 0, g, K, buf, err);
            else hipLaunchKernelGGL(k_barriers<1>, dim3(B), dim3(T), 0, 0, g, K, buf, err);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r) best = ms < best ? ms : best;
        }
        Bar hb;
        unsigned he;
        (void)hipMemcpy(&hb, g, sizeof(Bar), hipMemcpyDeviceToHost);
        (void)hipMemcpy(&he, err, sizeof(unsigned), hipMemcpyDeviceToHost);
        printf("mode %d: %d blocks x %d threads, %d barriers: %.2f us total, %.2f us per barrier (abort %u, data errors %u)\n",
               mode, B, T, 2 * K, best * 1e3f, best * 1e3f / (2 * K), hb.abort, he);
    }
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        (void)hipEventRecord(e0);
        for (int k = 0; k <= 2 * K; ++k) hipLaunchKernelGGL(k_empty, dim3(B), dim3(T), 0, 0, buf);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r) best = ms < best ? ms : best;
    }
    printf("dependent launches: %d back-to-back empty kernels (%d blocks): %.2f us total, %.2f us each\n", 2 * K + 1, B,
           best * 1e3f, best * 1e3f / (2 * K + 1));
    return 0;
}
