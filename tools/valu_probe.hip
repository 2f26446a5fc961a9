// valu_probe.hip -- diagnostic: the VALU / SALU / mixed issue ceilings of a CU at the occupancies the
// codec kernels run (one-wave workgroups, 4..32 per CU), to tell an issue-bound kernel from a
// latency-bound one.  Each wave runs independent integer chains; the kernel reports wave-instructions
// per CU-cycle (shader clock from s_memtime / s_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 -o valu_probe tools/valu_probe.hip && ./valu_probe
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

constexpr int kIters = 4096;

// 8 independent VALU chains, 8 VALU per iteration
__global__ __launch_bounds__(64) void valu_kernel(uint32_t* out, uint64_t* clk)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kIters; i++) {
        asm volatile(
            "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
            "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(i));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// 8 independent SALU chains (wave-uniform values)
__global__ __launch_bounds__(64) void salu_kernel(uint32_t* out, uint64_t* clk)
{
    uint32_t s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kIters; i++) {
        asm volatile(
            "s_add_u32 %0, %0, %8\n s_add_u32 %1, %1, %8\n s_add_u32 %2, %2, %8\n s_add_u32 %3, %3, %8\n"
            "s_add_u32 %4, %4, %8\n s_add_u32 %5, %5, %8\n s_add_u32 %6, %6, %8\n s_add_u32 %7, %7, %8\n"
            : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
            : "s"(i)
            : "scc");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// 4 VALU + 4 SALU chains interleaved
__global__ __launch_bounds__(64) void mixed_kernel(uint32_t* out, uint64_t* clk)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kIters; i++) {
        asm volatile(
            "v_add_u32 %0, %0, %8\n s_add_u32 %4, %4, %9\n v_add_u32 %1, %1, %8\n s_add_u32 %5, %5, %9\n"
            "v_add_u32 %2, %2, %8\n s_add_u32 %6, %6, %9\n v_add_u32 %3, %3, %8\n s_add_u32 %7, %7, %9\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
            : "v"(i), "s"(i)
            : "scc");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ s0 ^ s1 ^ s2 ^ s3;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    uint64_t* clk;
    const int maxBlocks = cus * 32;
    CHK(hipMalloc(&out, 4 * 64 * (size_t)maxBlocks));
    CHK(hipMalloc(&clk, 16 * (size_t)maxBlocks));
    uint64_t* h = (uint64_t*)malloc(16 * (size_t)maxBlocks);
    const char* names[3] = {"VALU", "SALU", "VALU+SALU"};
    for (int k = 0; k < 3; k++) {
        for (int per : {4, 8, 16, 20, 32}) {
            const int blocks = cus * per;
            hipEvent_t e0, e1;
            CHK(hipEventCreate(&e0));
            CHK(hipEventCreate(&e1));
            for (int rep = 0; rep < 2; rep++) {
                CHK(hipEventRecord(e0, 0));
                if (k == 0) hipLaunchKernelGGL(valu_kernel, dim3(blocks), dim3(64), 0, 0, out, clk);
                else if (k == 1) hipLaunchKernelGGL(salu_kernel, dim3(blocks), dim3(64), 0, 0, out, clk);
                else hipLaunchKernelGGL(mixed_kernel, dim3(blocks), dim3(64), 0, 0, out, clk);
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
            }
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(h, clk, 16 * (size_t)blocks, hipMemcpyDeviceToHost));
            double cyc = 0, real = 0;
            for (int b = 0; b < blocks; b++) {
                cyc += (double)h[2 * b];
                real += (double)h[2 * b + 1];
            }
            const double ghz = cyc / real * 0.1;  // s_memrealtime ticks at 100 MHz
            const double instrs = (double)blocks * kIters * 8.0;
            const double cuCycles = (double)cus * ms * 1e-3 * ghz * 1e9;
            printf("%-10s %2d waves/CU: %.3f ms, clock %.2f GHz, %.3f wave-instr per CU-cycle\n", names[k], per, ms, ghz,
                   instrs / cuCycles);
            CHK(hipEventDestroy(e0));
            CHK(hipEventDestroy(e1));
        }
    }
    return 0;
}
