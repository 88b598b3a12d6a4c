// FETCH_SIZE / WRITE_SIZE calibration for the access widths k_step's traffic is made of (development aid, VERDICT r5
// item 3).  MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16 B/lane streaming reads (it reports half the bytes
// there) and WRITE_SIZE for 16 B/lane stores; k_step's memory-side traffic is mostly the __noinline__ phases'
// callee-saved VGPR saves / restores -- dword scratch stores and loads, one 256-byte line segment per wave
// instruction.  This program moves a known byte count in each pattern, over a footprint far beyond L2 and the
// Infinity Cache, one kernel per pattern:
//   k_fill      16 B/lane stores, 2 GiB           (guide-calibrated: WRITE_SIZE = bytes)
//   k_wr4       4 B/lane stores (one dword per lane per instruction, coalesced), 2 GiB
//   k_rd16      16 B/lane loads of 2 GiB          (guide-calibrated: FETCH_SIZE = bytes / 2)
//   k_rd4       4 B/lane loads of 2 GiB
//   k_scratch   private-array traffic: every lane stores, then loads, SCR dwords of its own scratch (the compiler's
//               scratch_store_dword / scratch_load_dword, swizzled per lane: 256 B per wave instruction), with enough
//               waves in flight that the scratch footprint exceeds the Infinity Cache
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); the program prints each kernel's
// byte count.  tools/fetchcal.py divides.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/micro/fetchcal tools/micro/fetchcal.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_fill(uint4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}
__global__ void k_wr4(uint32_t* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i * 2654435761u;
}
__global__ void k_rd16(const uint4* p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) out[0] = acc; /* keeps the loads; almost never stores */
}
__global__ void k_rd4(const uint32_t* p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) out[0] = acc;
}
#define SCR 1024 /* dwords of scratch per lane: 4 KiB per lane, 256 KiB per wave */
__global__ void __launch_bounds__(64) k_scratch(const int* idx, uint32_t* out, int rounds) {
    /* a private array under run-time (wave-uniform) indices: it lives in scratch, every access a scratch_store_dword /
     * scratch_load_dword of the same index on all 64 lanes (the swizzled per-lane dword layout: 256 contiguous bytes),
     * the pattern of the callee-saved VGPR saves / restores */
    uint32_t buf[SCR];
    const int k = __builtin_amdgcn_readfirstlane(idx[0]);
    uint32_t acc = 0;
    for (int r = 0; r < rounds; r++) {
        for (int i = 0; i < SCR; i++) buf[(i * 7 + k) & (SCR - 1)] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(r + threadIdx.x);
        for (int i = 0; i < SCR; i++) acc += buf[(i * 13 + k) & (SCR - 1)];
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
    const size_t bytes = (size_t)2 << 30; /* 2 GiB: 8x the Infinity Cache */
    void* buf = nullptr;
    uint32_t* out = nullptr;
    int* idx = nullptr;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMalloc(&out, 4096 * sizeof(uint32_t)));
    CHK(hipMalloc(&idx, 8 * sizeof(int)));
    CHK(hipMemset(idx, 0, 8 * sizeof(int)));
    const int grid = 256 * 32, block = 256;
    const size_t n16 = bytes / 16, n4 = bytes / 4;
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(block), 0, 0, (uint4*)buf, n16);
    CHK(hipDeviceSynchronize());
    printf("k_fill    stores %zu B (16 B/lane)\n", bytes);
    hipLaunchKernelGGL(k_rd16, dim3(grid), dim3(block), 0, 0, (const uint4*)buf, n16, out);
    CHK(hipDeviceSynchronize());
    printf("k_rd16    loads  %zu B (16 B/lane)\n", bytes);
    hipLaunchKernelGGL(k_wr4, dim3(grid), dim3(block), 0, 0, (uint32_t*)buf, n4);
    CHK(hipDeviceSynchronize());
    printf("k_wr4     stores %zu B (4 B/lane)\n", bytes);
    hipLaunchKernelGGL(k_rd4, dim3(grid), dim3(block), 0, 0, (const uint32_t*)buf, n4, out);
    CHK(hipDeviceSynchronize());
    printf("k_rd4     loads  %zu B (4 B/lane)\n", bytes);
    /* scratch: 16,384 one-wave blocks x 256 KiB = 4 GiB stored and 4 GiB loaded per round; the in-flight footprint
     * (every wave slot of the chip at this kernel's occupancy) is several hundred MiB */
    const int sgrid = 16384, rounds = 1;
    hipLaunchKernelGGL(k_scratch, dim3(sgrid), dim3(64), 0, 0, idx, out, rounds);
    CHK(hipDeviceSynchronize());
    const size_t sb = (size_t)sgrid * 64 * SCR * 4 * rounds;
    printf("k_scratch stores %zu B, loads %zu B (4 B/lane scratch)\n", sb, sb);
    CHK(hipFree(buf));
    CHK(hipFree(out));
    CHK(hipFree(idx));
    return 0;
}
