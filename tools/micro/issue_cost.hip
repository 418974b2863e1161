// Issue cost of one wave64 vector instruction per class on gfx950, measured at wall clock.
//
// Each kernel issues U = 16 instructions of ONE class per loop iteration from inline asm
// (asm volatile: the compiler can neither drop, merge nor re-select them; tools/micro/
// issue_cost_check.py counts them in the compiled ISA and fails if the loop body holds
// anything else of that class), with no register dependency between them (8 destination
// registers, loop-invariant sources), so the figure is the SIMD's issue throughput for the
// class, not a latency. W waves per SIMD = W blocks of 256 threads per CU. Reported:
//   cyc = wall time x 2.4 GHz / (W x iters x U)     (SIMD-cycles per wave64 instruction)
// i.e. the cost in the units of the roofline's 1024 SIMDs x 2.4 GHz, DVFS included; the
// in-kernel shader clock (s_memtime vs the 100 MHz s_memrealtime) is printed beside it.
// The "mix" kinds interleave classes to check that costs add.
//
// usage: issue_cost [kind|all] [W ...]   (default: every kind at W = 1, 2, 4, 8)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f2v __attribute__((ext_vector_type(2)));

#define U16(X) X X X X X X X X X X X X X X X X

// destinations rotate over 8 registers per class; sources are loop-invariant
#define R8(T, name) T name##0 = 0, name##1 = 0, name##2 = 0, name##3 = 0, name##4 = 0, name##5 = 0, name##6 = 0, name##7 = 0

enum Kind {
    K_FMA_F64, K_MUL_F64, K_ADD_F64, K_FMA_F32, K_MUL_F32, K_PK_FMA_F32, K_PK_MUL_F32, K_ADD_U32, K_AND_B32,
    K_LSHL_ADD_U32, K_MOV_B32, K_MOV_B64, K_CNDMASK, K_CMP_F32, K_CMP_F64, K_MAD_U64, K_LSHL_ADD_U64, K_CVT_F32_F64,
    K_RSQ_F32, K_MIX_F64_PK, K_MIX_PK_INT, K_SALU, K_MIX_PK_SALU, K_MIX_PK_SALU_HALF, K_MIX_PK_DS, K_MIX_PK_CMP,
    K_FMAC_F32, K_ADD_F32, K_CMP_F32_VCC, K_CNDMASK_VCC, K_OR3_B32, K_PK_ADD_F32, K_MAX_F32, K_READFIRSTLANE,
    K_FMAC_F64, K_MBCNT_LO, K_LSHLREV_B64, K_BFE_U32, K_CVT_F64_F32, K_FMA_F32_BANKS, K_FMA_F32_SAMEBANK,
    K_PK_FMA_BANKS, K_PK_FMA_SAMEBANK, K_FMA_F64_BANKS, K_MIX_PK_SALU_DEP, K_NKIND
};
static const char *kind_name[] = {
    "v_fma_f64", "v_mul_f64", "v_add_f64", "v_fma_f32", "v_mul_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_add_u32",
    "v_and_b32", "v_lshl_add_u32", "v_mov_b32", "v_mov_b64", "v_cndmask_b32", "v_cmp_lt_f32", "v_cmp_lt_f64",
    "v_mad_u64_u32", "v_lshl_add_u64", "v_cvt_f32_f64", "v_rsq_f32", "mix:fma_f64+2pk_fma_f32",
    "mix:pk_fma_f32+add_u32", "s_add_u32", "mix:pk_fma_f32+s_add_u32", "mix:2pk_fma_f32+s_add_u32",
    "mix:2pk_fma_f32+ds_read_b64", "mix:pk_fma_f32+v_cmp_lt_f32", "v_fmac_f32_e32", "v_add_f32_e32",
    "v_cmp_lt_f32_e32", "v_cndmask_b32_e32", "v_or3_b32", "v_pk_add_f32", "v_max_f32_e32", "v_readfirstlane_b32",
    "v_fmac_f64_e32", "v_mbcnt_lo_u32_b32", "v_lshlrev_b64", "v_bfe_u32", "v_cvt_f64_f32",
    "v_fma_f32 (3 banks)", "v_fma_f32 (1 bank)", "v_pk_fma_f32 (3 banks)", "v_pk_fma_f32 (1 bank)",
    "v_fma_f64 (3 banks)", "mix:pk_fma_f32+s_cmp/s_cselect/s_and"};
// instructions per loop iteration (all classes)
static const int kind_u[] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 48, 32,
                             16, 32, 24, 24, 32, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16,
                             16, 16, 16, 16, 16, 64};

template <int KIND>
__global__ __launch_bounds__(256) void k_issue(float *out, unsigned long long *clk, int iters) {
    __shared__ double lds[512];
    lds[threadIdx.x] = threadIdx.x;
    lds[threadIdx.x + 256] = 0.5 * threadIdx.x;
    __syncthreads();
    const unsigned la = (unsigned)(uintptr_t)(lds + (threadIdx.x & 63));   // LDS byte address
    const float fs = threadIdx.x * 1e-3f + 1.0f;
    const double ds = threadIdx.x * 1e-3 + 1.0;
    const unsigned us = threadIdx.x * 7u + 3u;
    const f2v ps = {fs, fs + 1.0f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    R8(double, d);
    R8(float, f);
    R8(unsigned, u);
    f2v p0 = ps, p1 = ps, p2 = ps, p3 = ps, p4 = ps, p5 = ps, p6 = ps, p7 = ps;
    unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0, m6 = 0, m7 = 0;
#define ROT8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
    if constexpr (KIND >= K_FMA_F32_BANKS && KIND <= K_FMA_F64_BANKS)
        asm volatile("v_mov_b32 v40, 1.0\n\tv_mov_b32 v41, 1.0\n\tv_mov_b32 v42, 1.0\n\tv_mov_b32 v43, 1.0\n\t"
                     "v_mov_b32 v52, 1.0\n\tv_mov_b32 v53, 1.0\n\tv_mov_b32 v56, 1.0\n\tv_mov_b32 v57, 1.0\n\t"
                     "v_mov_b32 v58, 1.0\n\tv_mov_b32 v59, 1.0"
                     ::: "v40", "v41", "v42", "v43", "v52", "v53", "v56", "v57", "v58", "v59");
    for (int it = 0; it < iters; ++it) {
        if constexpr (KIND == K_FMA_F64) {
#define I(k) asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(d##k) : "v"(ds), "v"(ds), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MUL_F64) {
#define I(k) asm volatile("v_mul_f64 %0, %1, %2" : "+v"(d##k) : "v"(ds), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_ADD_F64) {
#define I(k) asm volatile("v_add_f64 %0, %1, %2" : "+v"(d##k) : "v"(ds), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_FMA_F32) {
#define I(k) asm volatile("v_fma_f32 %0, %1, %2, %3" : "+v"(f##k) : "v"(fs), "v"(fs), "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MUL_F32) {
#define I(k) asm volatile("v_mul_f32 %0, %1, %2" : "+v"(f##k) : "v"(fs), "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_PK_FMA_F32) {
#define I(k) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(p##k) : "v"(ps), "v"(ps), "v"(ps));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_PK_MUL_F32) {
#define I(k) asm volatile("v_pk_mul_f32 %0, %1, %2" : "+v"(p##k) : "v"(ps), "v"(ps));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_ADD_U32) {
#define I(k) asm volatile("v_add_u32 %0, %1, %2" : "+v"(u##k) : "v"(us), "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_AND_B32) {
#define I(k) asm volatile("v_and_b32 %0, %1, %2" : "+v"(u##k) : "v"(us), "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_LSHL_ADD_U32) {
#define I(k) asm volatile("v_lshl_add_u32 %0, %1, 3, %2" : "+v"(u##k) : "v"(us), "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MOV_B32) {
#define I(k) asm volatile("v_mov_b32 %0, %1" : "+v"(u##k) : "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MOV_B64) {
#define I(k) asm volatile("v_mov_b64 %0, %1" : "+v"(d##k) : "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_CNDMASK) {
            // the lane mask comes from a scalar register pair (the kernels' ballot masks)
#define I(k) asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "+v"(u##k) : "v"(us), "v"(us), "s"(0x5555555555555555ull));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_CMP_F32) {
#define I(k) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "+s"(m##k) : "v"(fs), "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_CMP_F64) {
#define I(k) asm volatile("v_cmp_lt_f64_e64 %0, %1, %2" : "+s"(m##k) : "v"(ds), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MAD_U64) {
#define I(k) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "+v"(d##k), "=s"(m##k) : "v"(us), "v"(us), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_LSHL_ADD_U64) {
#define I(k) asm volatile("v_lshl_add_u64 %0, %1, 3, %2" : "+v"(d##k) : "v"(ds), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_CVT_F32_F64) {
#define I(k) asm volatile("v_cvt_f32_f64 %0, %1" : "+v"(f##k) : "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_RSQ_F32) {
#define I(k) asm volatile("v_rsq_f32 %0, %1" : "+v"(f##k) : "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MIX_F64_PK) {
            // per iteration: 16 v_fma_f64 + 32 v_pk_fma_f32, interleaved 1:2
#define I(k) asm volatile("v_fma_f64 %0, %1, %2, %3" : "+v"(d##k) : "v"(ds), "v"(ds), "v"(ds)); \
             asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(p##k) : "v"(ps), "v"(ps), "v"(ps)); \
             asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(p##k) : "v"(ps), "v"(ps), "v"(ps));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_SALU) {
            // scalar ALU alone (separate issue port); one asm block, so no hazard padding between
#define SA(a, b) "s_add_u32 %" #a ", %" #a ", %" #b "\n\t"
            asm volatile(SA(0, 8) SA(1, 9) SA(2, 8) SA(3, 9) SA(4, 8) SA(5, 9) SA(6, 8) SA(7, 9)
                         SA(0, 9) SA(1, 8) SA(2, 9) SA(3, 8) SA(4, 9) SA(5, 8) SA(6, 9) SA(7, 8)
                         : "+s"(u0), "+s"(u1), "+s"(u2), "+s"(u3), "+s"(u4), "+s"(u5), "+s"(u6), "+s"(u7)
                         : "s"(3u), "s"(7u) : "scc");
        } else if constexpr (KIND == K_MIX_PK_SALU) {
            // one wave's stream of 16 v_pk_fma_f32 + 16 s_add_u32, interleaved 1:1 (one asm block)
#define PK(d) "v_pk_fma_f32 %" #d ", %10, %10, %10\n\t"
            asm volatile(PK(8) SA(0, 11) PK(9) SA(1, 11) PK(8) SA(2, 11) PK(9) SA(3, 11)
                         PK(8) SA(4, 11) PK(9) SA(5, 11) PK(8) SA(6, 11) PK(9) SA(7, 11)
                         PK(8) SA(0, 11) PK(9) SA(1, 11) PK(8) SA(2, 11) PK(9) SA(3, 11)
                         PK(8) SA(4, 11) PK(9) SA(5, 11) PK(8) SA(6, 11) PK(9) SA(7, 11)
                         : "+s"(u0), "+s"(u1), "+s"(u2), "+s"(u3), "+s"(u4), "+s"(u5), "+s"(u6), "+s"(u7),
                           "+v"(p0), "+v"(p1)
                         : "v"(ps), "s"(7u) : "scc");
        } else if constexpr (KIND == K_MIX_PK_SALU_HALF) {
            // 16 v_pk_fma_f32 + 8 s_add_u32 (the dominant kernel's hot loop holds ~0.6 SALU per VALU)
            asm volatile(PK(8) PK(9) SA(0, 11) PK(8) PK(9) SA(1, 11) PK(8) PK(9) SA(2, 11) PK(8) PK(9) SA(3, 11)
                         PK(8) PK(9) SA(4, 11) PK(8) PK(9) SA(5, 11) PK(8) PK(9) SA(6, 11) PK(8) PK(9) SA(7, 11)
                         : "+s"(u0), "+s"(u1), "+s"(u2), "+s"(u3), "+s"(u4), "+s"(u5), "+s"(u6), "+s"(u7),
                           "+v"(p0), "+v"(p1)
                         : "v"(ps), "s"(7u) : "scc");
        } else if constexpr (KIND == K_MIX_PK_DS) {
            // 16 v_pk_fma_f32 + 8 ds_read_b64 (LDS operand reads of the sweep), drained per iteration
#define I(k) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(p##k) : "v"(ps), "v"(ps), "v"(ps)); \
             asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(p##k) : "v"(ps), "v"(ps), "v"(ps)); \
             asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(d##k) : "v"(la), "i"(8 * k));
            ROT8(I)
#undef I
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if constexpr (KIND == K_MIX_PK_CMP) {
            // 16 v_pk_fma_f32 + 16 v_cmp_lt_f32 (to SGPR pairs): the sweep's decision compares
#define I(k) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(p##k) : "v"(ps), "v"(ps), "v"(ps)); \
             asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "+s"(m##k) : "v"(fs), "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_FMAC_F32) {
#define I(k) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(f##k) : "v"(fs), "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_ADD_F32) {
#define I(k) asm volatile("v_add_f32_e32 %0, %1, %2" : "+v"(f##k) : "v"(fs), "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_CMP_F32_VCC) {
#define I(k) asm volatile("v_cmp_lt_f32_e32 vcc, %0, %1" : : "v"(fs), "v"(f##k) : "vcc");
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_CNDMASK_VCC) {
#define I(k) asm volatile("v_cndmask_b32_e32 %0, %1, %2, vcc" : "+v"(u##k) : "v"(us), "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_OR3_B32) {
#define I(k) asm volatile("v_or3_b32 %0, %1, %2, %3" : "+v"(u##k) : "v"(us), "v"(us), "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_PK_ADD_F32) {
#define I(k) asm volatile("v_pk_add_f32 %0, %1, %2" : "+v"(p##k) : "v"(ps), "v"(ps));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MAX_F32) {
#define I(k) asm volatile("v_max_f32_e32 %0, %1, %2" : "+v"(f##k) : "v"(fs), "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_READFIRSTLANE) {
#define I(k) asm volatile("v_readfirstlane_b32 %0, %1" : "+s"(u##k) : "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_FMAC_F64) {
#define I(k) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(d##k) : "v"(ds), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MBCNT_LO) {
#define I(k) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, %1" : "+v"(u##k) : "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_LSHLREV_B64) {
#define I(k) asm volatile("v_lshlrev_b64 %0, %1, %2" : "+v"(d##k) : "v"(us), "v"(ds));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_BFE_U32) {
#define I(k) asm volatile("v_bfe_u32 %0, %1, %2, %3" : "+v"(u##k) : "v"(us), "v"(us), "v"(us));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_CVT_F64_F32) {
#define I(k) asm volatile("v_cvt_f64_f32_e32 %0, %1" : "+v"(d##k) : "v"(fs));
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_FMA_F32_BANKS) {
            // sources in three different VGPR banks (v40, v41, v42; bank = index mod 4),
            // destinations v44..v51 (explicit registers, declared clobbered)
#define I(k) asm volatile("v_fma_f32 v%0, v40, v41, v42" : : "i"(44 + k) : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_FMA_F32_SAMEBANK) {
            // all three sources in bank 0 (v40, v44 wait: v40, v52, v56)
#define I(k) asm volatile("v_fma_f32 v%0, v40, v52, v56" : : "i"(44 + k) : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_PK_FMA_BANKS) {
            // 64-bit pairs v[40:41], v[42:43], v[58:59]: banks {0,1} {2,3} {2,3}
#define I(k) asm volatile("v_pk_fma_f32 v[%0:%1], v[40:41], v[42:43], v[58:59]" : : "i"(44 + 2 * (k % 4)), "i"(45 + 2 * (k % 4)) : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_PK_FMA_SAMEBANK) {
#define I(k) asm volatile("v_pk_fma_f32 v[%0:%1], v[40:41], v[52:53], v[56:57]" : : "i"(44 + 2 * (k % 4)), "i"(45 + 2 * (k % 4)) : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_FMA_F64_BANKS) {
#define I(k) asm volatile("v_fma_f64 v[%0:%1], v[40:41], v[42:43], v[58:59]" : : "i"(44 + 2 * (k % 4)), "i"(45 + 2 * (k % 4)) : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
            ROT8(I) ROT8(I)
#undef I
        } else if constexpr (KIND == K_MIX_PK_SALU_DEP) {
            // the hot loop's shape: per packed FMA three dependent scalar ops (compare, select,
            // and-not) on SGPR pairs, as the per-candidate mask bookkeeping does (one asm block)
#define SD(m) "s_cmp_lg_u32 %4, %5\n\ts_cselect_b64 %" #m ", %" #m ", 0\n\ts_andn2_b64 %" #m ", %" #m ", %6\n\t"
#define PK2(d) "v_pk_fma_f32 %" #d ", %7, %7, %7\n\t"
            asm volatile(PK2(2) SD(0) PK2(3) SD(1) PK2(2) SD(0) PK2(3) SD(1) PK2(2) SD(0) PK2(3) SD(1)
                         PK2(2) SD(0) PK2(3) SD(1) PK2(2) SD(0) PK2(3) SD(1) PK2(2) SD(0) PK2(3) SD(1)
                         PK2(2) SD(0) PK2(3) SD(1) PK2(2) SD(0) PK2(3) SD(1)
                         : "+s"(m0), "+s"(m1), "+v"(p0), "+v"(p1)
                         : "s"(3u), "s"(7u), "s"(0x5555ull), "v"(ps) : "scc");
        } else if constexpr (KIND == K_MIX_PK_INT) {
            // per iteration: 16 v_pk_fma_f32 + 16 v_add_u32, interleaved 1:1
#define I(k) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "+v"(p##k) : "v"(ps), "v"(ps), "v"(ps)); \
             asm volatile("v_add_u32 %0, %1, %2" : "+v"(u##k) : "v"(us), "v"(us));
            ROT8(I) ROT8(I)
#undef I
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    // keep every destination live past the loop
    double s = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7;
    s += f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
    s += (double)(u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7);
    const f2v ps8 = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7;
    s += ps8[0] + ps8[1] + (double)((m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7) & 1ull);
    if (s == 12345.678) out[threadIdx.x] = (float)s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int KIND>
static void launch(int blocks, float *out, unsigned long long *clk, int iters) {
    hipLaunchKernelGGL(k_issue<KIND>, dim3(blocks), dim3(256), 0, 0, out, clk, iters);
}

typedef void (*launch_fn)(int, float *, unsigned long long *, int);
template <int... K>
static std::vector<launch_fn> table(std::integer_sequence<int, K...>) {
    return {&launch<K>...};
}

int main(int argc, char **argv) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    const auto fns = table(std::make_integer_sequence<int, K_NKIND>{});
    int k_lo = 0, k_hi = K_NKIND;
    if (argc > 1 && strcmp(argv[1], "all") != 0) {
        k_lo = atoi(argv[1]);
        k_hi = k_lo + 1;
    }
    std::vector<int> ws;
    for (int i = 2; i < argc; ++i) ws.push_back(atoi(argv[i]));
    if (ws.empty()) ws = {1, 2, 4, 8};
    float *out;
    unsigned long long *clk, hc[2];
    if (hipMalloc(&out, 1024 * sizeof(float)) != hipSuccess || hipMalloc(&clk, 16) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    printf("{\"cus\": %d, \"clock_mhz\": %.0f, \"rows\": [\n", cus, p.clockRate / 1e3);
    bool first = true;
    for (int k = k_lo; k < k_hi; ++k) {
        for (int W : ws) {
            // ~2-4 ms per launch: iterations scaled so each SIMD issues ~4e6 instruction-cycles
            const int iters = (int)(2.0e5 / (double)(W * kind_u[k]) * 16.0);
            float ms = 0.0f, best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0);
                fns[k](cus * W, out, clk, iters);
                (void)hipEventRecord(e1);
                if (hipEventSynchronize(e1) != hipSuccess) return 2;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (rep > 0 && ms < best) best = ms;
            }
            if (hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost) != hipSuccess) return 3;
            const double instr = (double)W * iters * kind_u[k];                  // per SIMD
            const double cyc = best * 1e-3 * 2.4e9 / instr;
            const double ghz = (double)hc[0] / ((double)hc[1] / 100e6) / 1e9;
            const double cyc_clk = best * 1e-3 * ghz * 1e9 / instr;
            printf("%s {\"kind\": %d, \"name\": \"%s\", \"waves_per_simd\": %d, \"iters\": %d, \"per_iter\": %d, "
                   "\"ms\": %.4f, \"cyc_at_2p4\": %.3f, \"shader_ghz\": %.3f, \"cyc_at_shader_clock\": %.3f}",
                   first ? "" : ",\n", k, kind_name[k], W, iters, kind_u[k], best, cyc, ghz, cyc_clk);
            first = false;
            fflush(stdout);
        }
    }
    printf("\n]}\n");
    return 0;
}
