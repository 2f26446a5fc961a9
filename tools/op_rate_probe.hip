// op_rate_probe.hip -- diagnostic: the issue rate of single VALU opcodes the merge / split / Huffman
// inner loops are built from (v_perm_b32, v_mad_u32_u24, 64-bit shifts and adds, packed 16-bit ops,
// ...), as wave-instructions per CU-cycle at 16 one-wave workgroups per CU, 8 independent chains per
// wave.  A full-rate opcode reads ~1.0 (four SIMDs, a wave64 VALU op every 4 cycles each).
//   hipcc --offload-arch=gfx950 -O3 -o op_rate_probe tools/op_rate_probe.hip && ./op_rate_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e));                             \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

constexpr int kIters = 8192;

// 8 independent 32-bit chains: "OP %k, %k, src..." with the operand list given by ARGS
#define PROBE32(NAME, OP, ARGS)                                                                         \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, uint64_t* clk)                            \
    {                                                                                                   \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
                 a6 = a0 + 6, a7 = a0 + 7;                                                              \
        uint32_t b = threadIdx.x * 3u + 1u;                                                             \
        const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();       \
        for (int i = 0; i < kIters; i++) {                                                              \
            asm volatile(OP " %0, %0, " ARGS "\n " OP " %1, %1, " ARGS "\n " OP " %2, %2, " ARGS "\n "      \
                         OP " %3, %3, " ARGS "\n " OP " %4, %4, " ARGS "\n " OP " %5, %5, " ARGS "\n "      \
                         OP " %6, %6, " ARGS "\n " OP " %7, %7, " ARGS "\n"                                \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(b));                                                                     \
        }                                                                                               \
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();       \
        out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                     \
        if (threadIdx.x == 0) {                                                                         \
            clk[2 * blockIdx.x] = t1 - t0;                                                              \
            clk[2 * blockIdx.x + 1] = r1 - r0;                                                          \
        }                                                                                               \
    }

// 8 independent 64-bit chains
#define PROBE64(NAME, OP, ARGS)                                                                         \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, uint64_t* clk)                            \
    {                                                                                                   \
        uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
                 a6 = a0 + 6, a7 = a0 + 7;                                                              \
        uint64_t b = threadIdx.x * 3u + 1u;                                                             \
        uint32_t s = threadIdx.x & 31u;                                                                 \
        const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();       \
        for (int i = 0; i < kIters; i++) {                                                              \
            asm volatile(OP " %0, " ARGS "\n " OP " %1, " ARGS "\n " OP " %2, " ARGS "\n "                  \
                         OP " %3, " ARGS "\n " OP " %4, " ARGS "\n " OP " %5, " ARGS "\n "                  \
                         OP " %6, " ARGS "\n " OP " %7, " ARGS "\n"                                        \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(b), "v"(s));                                                             \
        }                                                                                               \
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();       \
        out[blockIdx.x * 64 + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);        \
        if (threadIdx.x == 0) {                                                                         \
            clk[2 * blockIdx.x] = t1 - t0;                                                              \
            clk[2 * blockIdx.x + 1] = r1 - r0;                                                          \
        }                                                                                               \
    }

PROBE32(p_add, "v_add_u32", "%8")
PROBE32(p_perm, "v_perm_b32", "%8, %8")
PROBE32(p_mad24, "v_mad_u32_u24", "%8, %8")
PROBE32(p_bfe, "v_bfe_u32", "%8, 3")
PROBE32(p_bfi, "v_bfi_b32", "%8, %8")
PROBE32(p_min3, "v_min3_u32", "%8, %8")
PROBE32(p_bcnt, "v_bcnt_u32_b32", "%8")
PROBE32(p_lshl_add, "v_lshl_add_u32", "4, %8")
PROBE32(p_pk_add, "v_pk_add_u16", "%8")
PROBE32(p_alignbit, "v_alignbit_b32", "%8, %8")
PROBE32(p_mul_lo, "v_mul_lo_u32", "%8")
PROBE32(p_and, "v_and_b32", "%8")
PROBE32(p_xor, "v_xor_b32", "%8")
PROBE32(p_lshl, "v_lshlrev_b32", "%8")
PROBE32(p_lshr, "v_lshrrev_b32", "%8")
PROBE32(p_max, "v_max_u32", "%8")
PROBE32(p_mul24, "v_mul_u32_u24", "%8")
PROBE32(p_add_e64, "v_add_u32_e64", "%8")
PROBE32(p_add_sdwa, "v_add_u32_sdwa", "%8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")
// alternating VOP2 add / VOP3 perm (4 + 4)
__global__ __launch_bounds__(64) void p_mix(uint32_t* out, uint64_t* clk)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t b = threadIdx.x * 3u + 1u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kIters; i++) {
        asm volatile("v_add_u32 %0, %0, %8\n v_perm_b32 %1, %1, %8, %8\n v_add_u32 %2, %2, %8\n v_perm_b32 %3, %3, %8, %8\n"
                     "v_add_u32 %4, %4, %8\n v_perm_b32 %5, %5, %8, %8\n v_add_u32 %6, %6, %8\n v_perm_b32 %7, %7, %8, %8\n"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}
// 64-bit: dst is the chain register, operands ARGS (%8 = 64-bit b, %9 = 32-bit shift)
PROBE64(p_lshl64, "v_lshlrev_b64", "%9, %0")
PROBE64(p_lshl_add64, "v_lshl_add_u64", "%0, 0, %8")

typedef void (*Kern)(uint32_t*, uint64_t*);
int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int per = 16;
    const int blocks = cus * per;
    uint32_t* out;
    uint64_t* clk;
    CHK(hipMalloc(&out, 4 * 64 * (size_t)blocks));
    CHK(hipMalloc(&clk, 16 * (size_t)blocks));
    uint64_t* h = (uint64_t*)malloc(16 * (size_t)blocks);
    struct {
        const char* name;
        Kern k;
        double opsPerSlot;  // instructions per asm slot
    } probes[] = {
        {"v_add_u32", p_add, 1},           {"v_perm_b32", p_perm, 1},         {"v_mad_u32_u24", p_mad24, 1},
        {"v_bfe_u32", p_bfe, 1},           {"v_bfi_b32", p_bfi, 1},           {"v_min3_u32", p_min3, 1},
        {"v_bcnt_u32_b32", p_bcnt, 1},     {"v_lshl_add_u32", p_lshl_add, 1}, {"v_pk_add_u16", p_pk_add, 1},
        {"v_alignbit_b32", p_alignbit, 1}, {"v_mul_lo_u32", p_mul_lo, 1},     {"v_lshlrev_b64", p_lshl64, 1},
        {"v_lshl_add_u64", p_lshl_add64, 1},
        {"v_and_b32", p_and, 1},           {"v_xor_b32", p_xor, 1},           {"v_lshlrev_b32", p_lshl, 1},
        {"v_lshrrev_b32", p_lshr, 1},      {"v_max_u32", p_max, 1},           {"v_mul_u32_u24", p_mul24, 1},
        {"v_add_u32_e64 (VOP3)", p_add_e64, 1}, {"v_add_u32_sdwa", p_add_sdwa, 1},
        {"v_add_u32 / v_perm_b32 mix", p_mix, 1},
        {"v_add_u32 (again)", p_add, 1},
    };
    for (auto& pr : probes) {
        hipEvent_t e0, e1;
        CHK(hipEventCreate(&e0));
        CHK(hipEventCreate(&e1));
        float ms = 0;
        for (int rep = 0; rep < 3; rep++) {
            CHK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(pr.k, dim3(blocks), dim3(64), 0, 0, out, clk);
            CHK(hipGetLastError());
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
        }
        CHK(hipEventElapsedTime(&ms, e0, e1));
        CHK(hipMemcpy(h, clk, 16 * (size_t)blocks, hipMemcpyDeviceToHost));
        double cyc = 0, real = 0;
        for (int b = 0; b < blocks; b++) {
            cyc += (double)h[2 * b];
            real += (double)h[2 * b + 1];
        }
        const double ghz = cyc / real * 0.1;  // s_memrealtime ticks at 100 MHz
        const double instrs = (double)blocks * kIters * 8.0 * pr.opsPerSlot;
        const double cuCycles = (double)cus * ms * 1e-3 * ghz * 1e9;
        printf("%-28s %.3f ms, clock %.2f GHz, %.3f wave-instr per CU-cycle\n", pr.name, ms, ghz, instrs / cuCycles);
        CHK(hipEventDestroy(e0));
        CHK(hipEventDestroy(e1));
    }
    return 0;
}
