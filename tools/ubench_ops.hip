// Microbenchmark: issue cost of the integer VALU / SALU instructions the route kernel could use,
// on gfx950. Each kernel runs ITER rounds of 8 independent instances of one instruction per wave
// (inline asm, so the instruction is exactly the one named). The grid fills every SIMD with
// WAVES_PER_SIMD waves; the in-kernel clock comes from s_memtime / s_memrealtime (100 MHz).
// Output: one JSON line, per op the SIMD cycles per wave-instruction (throughput, all waves).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_ops tools/ubench_ops.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITER = 2048;
constexpr int kBlock = 256;

#define BODY8(INS)                                                                              \
    asm volatile(INS : "+v"(a0) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(a1) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(a2) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(a3) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(a4) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(a5) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(a6) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(a7) : "v"(b0), "v"(c0) : "vcc", "scc");

#define BODY8_64(INS)                                                                           \
    asm volatile(INS : "+v"(q0) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(q1) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(q2) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(q3) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(q4) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(q5) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(q6) : "v"(b0), "v"(c0) : "vcc", "scc");                                           \
    asm volatile(INS : "+v"(q7) : "v"(b0), "v"(c0) : "vcc", "scc");

#define BODY8_S(INS)                                                                            \
    asm volatile(INS : "+s"(s0) : "s"(t0) : "scc");                                                    \
    asm volatile(INS : "+s"(s1) : "s"(t0) : "scc");                                                    \
    asm volatile(INS : "+s"(s2) : "s"(t0) : "scc");                                                    \
    asm volatile(INS : "+s"(s3) : "s"(t0) : "scc");                                                    \
    asm volatile(INS : "+s"(s4) : "s"(t0) : "scc");                                                    \
    asm volatile(INS : "+s"(s5) : "s"(t0) : "scc");                                                    \
    asm volatile(INS : "+s"(s6) : "s"(t0) : "scc");                                                    \
    asm volatile(INS : "+s"(s7) : "s"(t0) : "scc");

template <int OP>
__global__ __launch_bounds__(kBlock) void kern(uint32_t seed, uint64_t *out, uint64_t *clk) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    uint32_t b0 = seed * 3 + threadIdx.x, c0 = seed ^ 0x5A5A5A5Au;
    uint64_t q0 = a0, q1 = a1, q2 = a2, q3 = a3, q4 = a4, q5 = a5, q6 = a6, q7 = a7;
    uint32_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3, s4 = seed + 4, s5 = seed + 5, s6 = seed + 6,
             s7 = seed + 7, t0 = blockIdx.x;
    typedef int v4i __attribute__((ext_vector_type(4)));
    v4i acc0 = {(int)a0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    v4i xa = {(int)b0, (int)c0, 1, 2}, xb = {(int)c0, 3, (int)b0, 4};
    const uint64_t m0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITER; ++it) {
        if (OP == 0) { BODY8("v_add_u32 %0, %1, %0") }
        if (OP == 1) { BODY8("v_xor_b32 %0, %1, %0") }
        if (OP == 2) { BODY8("v_mul_lo_u32 %0, %1, %0") }
        if (OP == 3) { BODY8("v_mul_hi_u32 %0, %1, %0") }
        if (OP == 4) { BODY8_64("v_mad_u64_u32 %0, vcc, %1, %2, %0") }
        if (OP == 5) { BODY8("v_mul_u32_u24 %0, %1, %0") }
        if (OP == 6) { BODY8("v_mad_u32_u24 %0, %1, %2, %0") }
        if (OP == 7) { BODY8("v_dot4_i32_i8 %0, %1, %2, %0") }
        if (OP == 8) { BODY8("v_dot4_u32_u8 %0, %1, %2, %0") }
        if (OP == 9) { BODY8("v_perm_b32 %0, %1, %2, %0") }
        if (OP == 10) { BODY8("v_alignbyte_b32 %0, %1, %2, %0") }
        if (OP == 11) { BODY8_64("v_lshlrev_b64 %0, 6, %0") }
        if (OP == 12) { BODY8_64("v_lshl_add_u64 %0, %0, 6, %0") }
        if (OP == 13) { BODY8("v_bfe_i32 %0, %0, 8, 8") }
        if (OP == 14) { BODY8("v_mul_hi_u32_u24 %0, %1, %0") }
        if (OP == 15) { BODY8("v_add3_u32 %0, %1, %2, %0") }
        if (OP == 16) { BODY8("v_and_or_b32 %0, %1, %2, %0") }
        if (OP == 17) { BODY8("v_lshl_or_b32 %0, %1, 3, %0") }
        if (OP == 18) { BODY8("v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:BYTE_1 src1_sel:DWORD") }
        if (OP == 19) { BODY8_S("s_add_u32 %0, %1, %0") }
        if (OP == 20) { BODY8_S("s_lshl_b32 %0, %0, 1") }
        if (OP == 21) { BODY8("v_cndmask_b32 %0, %1, %0, vcc") }
        if (OP == 22) { BODY8("v_bfi_b32 %0, %1, %2, %0") }
        if (OP == 23) { BODY8("v_mad_i32_i24 %0, %1, %2, %0") }
        if (OP == 24) { BODY8("v_dot2_i32_i16 %0, %1, %2, %0") }
        if (OP == 25) { BODY8("v_pk_mad_u16 %0, %1, %2, %0") }
        if (OP == 26) { BODY8("v_xad_u32 %0, %1, %2, %0") }
        if (OP == 27) { BODY8_64("v_mad_i64_i32 %0, vcc, %1, %2, %0") }
        if (OP == 28) { BODY8("v_sad_u32 %0, %1, %2, %0") }
        if (OP == 29) { BODY8("v_msad_u8 %0, %1, %2, %0") }
        if (OP == 30) { BODY8("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:0") }
        if (OP == 31) { BODY8("v_add_co_u32 %0, vcc, %0, %1") }
        if (OP == 32) { BODY8("v_ffbl_b32 %0, %0") }
        if (OP == 33) { BODY8("v_bcnt_u32_b32 %0, %0, %1") }
        if (OP == 34) { BODY8_64("v_lshrrev_b64 %0, 6, %0") }
        if (OP == 35) { BODY8_64("v_mov_b64 %0, %0") }
        if (OP == 36) { BODY8("v_and_b32 %0, %1, %0") }
        if (OP == 37) { BODY8("v_or_b32 %0, %1, %0") }
        if (OP == 38) { BODY8("v_sub_u32 %0, %1, %0") }
        if (OP == 39) { BODY8("v_lshlrev_b32 %0, 3, %0") }
        if (OP == 40) { BODY8("v_lshrrev_b32 %0, 3, %0") }
        if (OP == 41) { BODY8("v_not_b32 %0, %0") }
        if (OP == 42) { BODY8("v_max_u32 %0, %1, %0") }
        if (OP == 43) { BODY8("v_cmp_eq_u32 vcc, %0, %1") }
        if (OP == 44) { BODY8("v_cndmask_b32_e64 %0, %1, %0, s[20:21]") }
        if (OP == 45) { BODY8("v_addc_co_u32 %0, vcc, %0, %1, vcc") }
        if (OP == 46) { BODY8("v_pk_add_u16 %0, %1, %0") }
        if (OP == 47) { BODY8("v_mad_u32_u16 %0, %1, %2, %0") }
        if (OP == 48) { BODY8("v_add_f32 %0, %1, %0") }
        if (OP == 49) { BODY8("v_fma_f32 %0, %1, %2, %0") }
        if (OP == 50) { BODY8("v_and_b32 %0, 0x7f7f7f7f, %0") }
        if (OP == 51) { BODY8("v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD") }
        if (OP == 52) { BODY8("v_mul_lo_u16 %0, %1, %0") }
        if (OP == 53) { BODY8("v_pk_mul_lo_u16 %0, %1, %0") }
        if (OP == 54) { BODY8("v_sub_co_u32 %0, vcc, %1, %0") }
        if (OP == 55) { BODY8("v_bfrev_b32 %0, %0") }
        if (OP == 56) { BODY8("v_lshl_add_u32 %0, %1, 2, %0") }
        if (OP == 57) { BODY8("v_xor_b32 %0, 0x0a0a0a0a, %0") }
        if (OP == 58) { BODY8("v_mov_b32 %0, %1") }
        if (OP == 59) { BODY8_64("v_pk_fma_f32 %0, %0, %0, %0") }
        if (OP == 60) { asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc0) : "v"(xa), "v"(xb)); asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc1) : "v"(xa), "v"(xb)); asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc2) : "v"(xa), "v"(xb)); asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc3) : "v"(xa), "v"(xb)); asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc0) : "v"(xa), "v"(xb)); asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc1) : "v"(xa), "v"(xb)); asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc2) : "v"(xa), "v"(xb)); asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc3) : "v"(xa), "v"(xb)); }
    }
    const uint64_t m1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * kBlock + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) ^ q0 ^ q1 ^ q2 ^ q3 ^
                                             q4 ^ q5 ^ q6 ^ q7 ^ (uint64_t)(acc0[0] ^ acc1[1] ^ acc2[2] ^ acc3[3]) ^ s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = m1 - m0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static const char *kNames[] = {
    "v_add_u32", "v_xor_b32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mul_u32_u24", "v_mad_u32_u24",
    "v_dot4_i32_i8", "v_dot4_u32_u8", "v_perm_b32", "v_alignbyte_b32", "v_lshlrev_b64", "v_lshl_add_u64",
    "v_bfe_i32", "v_mul_hi_u32_u24", "v_add3_u32", "v_and_or_b32", "v_lshl_or_b32", "v_cmp_eq_u32_sdwa",
    "s_add_u32", "s_lshl_b32", "v_cndmask_b32", "v_bfi_b32", "v_mad_i32_i24", "v_dot2_i32_i16", "v_pk_mad_u16",
    "v_xad_u32", "v_mad_i64_i32", "v_sad_u32", "v_msad_u8", "v_mov_b32_dpp", "v_add_co_u32", "v_ffbl_b32",
    "v_bcnt_u32_b32", "v_lshrrev_b64", "v_mov_b64", "v_and_b32", "v_or_b32", "v_sub_u32", "v_lshlrev_b32", "v_lshrrev_b32", "v_not_b32", "v_max_u32", "v_cmp_eq_u32_e32", "v_cndmask_b32_e64", "v_addc_co_u32", "v_pk_add_u16", "v_mad_u32_u16", "v_add_f32", "v_fma_f32", "v_and_b32_lit", "v_add_u32_sdwa", "v_mul_lo_u16", "v_pk_mul_lo_u16", "v_sub_co_u32_e32", "v_bfrev_b32", "v_lshl_add_u32", "v_xor_b32_lit", "v_mov_b32", "v_pk_fma_f32", "v_mfma_i32_16x16x64_i8"};

template <int OP>
void run(int blocks, uint64_t *out, uint64_t *clk, uint64_t *hclk, int first) {
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(kBlock), 0, 0, 1u, out, clk);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(kBlock), 0, 0, 2u, out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(hclk, clk, 2 * blocks * sizeof(uint64_t), hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int i = 0; i < blocks; ++i) {
        cyc += (double)hclk[2 * i];
        rt += (double)hclk[2 * i + 1];
    }
    const double ghz = cyc / rt / 10.0;   // memrealtime ticks at 100 MHz
    // every SIMD holds blocks*4/1024 waves; each wave issues ITER*8 instances
    const double waves_per_simd = blocks * (kBlock / 64) / 1024.0;
    const double cyc_per_inst = (ms * 1e-3) * ghz * 1e9 / (waves_per_simd * ITER * 8.0);
    printf("%s\"%s\": [%.2f, %.2f]", first ? "" : ", ", kNames[OP], cyc_per_inst, ghz);
    fflush(stdout);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

template <int... OPS>
void run_all(int blocks, uint64_t *out, uint64_t *clk, uint64_t *hclk, std::integer_sequence<int, OPS...>) {
    int first = 1;
    ((run<OPS>(blocks, out, clk, hclk, first), first = 0), ...);
}

int main() {
    const int blocks = 256 * 8;   // 8 waves per SIMD (4 waves per block, 256 CUs)
    uint64_t *out, *clk;
    hipMalloc(&out, (size_t)blocks * kBlock * 8);
    hipMalloc(&clk, (size_t)blocks * 16);
    static uint64_t hclk[2 * 256 * 8];
    printf("{\"cycles_per_wave_inst_and_ghz\": {");
    run_all(blocks, out, clk, hclk, std::make_integer_sequence<int, 61>{});
    printf("}}\n");
    return 0;
}
