// Latency of dependent FP64 chains in one wavefront (gfx950): cycles per step for
// v_add_f64, DPP-mov+add (reduce16 level), permlane32_swap broadcast, v_readlane, LDS read.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, false);
    int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double pl32(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double rl(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l), __builtin_amdgcn_readlane(__double2loint(x), l));
}
#define N 256
__device__ __forceinline__ unsigned long long tick(double& x) {
    unsigned long long t;
    int tmp, lo = __double2loint(x);
    asm volatile("v_readfirstlane_b32 %1, %2\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "=s"(tmp) : "v"(lo));
    asm volatile("" : "+v"(x));
    return t;
}
__global__ void k(double* out, unsigned long long* cyc, double seed, const double* yin) {
    __shared__ double lds[64];
    double x = seed + threadIdx.x, y = yin[threadIdx.x];
    lds[threadIdx.x] = x;
    __syncthreads();
    unsigned long long t0, t1;
    // 0: dependent add
    t0 = tick(x);
#pragma unroll
    for (int i = 0; i < N; i++) x = x + y;
    t1 = tick(x);
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    // 1: dependent mul
    t0 = tick(x);
#pragma unroll
    for (int i = 0; i < N; i++) x = x * y;
    t1 = tick(x);
    if (threadIdx.x == 0) cyc[1] = t1 - t0;
    // 2: dpp level
    t0 = tick(x);
#pragma unroll
    for (int i = 0; i < N; i++) x = x + dpp<0xB1>(x);
    t1 = tick(x);
    if (threadIdx.x == 0) cyc[2] = t1 - t0;
    // 3: permlane32 broadcast + add
    t0 = tick(x);
#pragma unroll
    for (int i = 0; i < N; i++) x = x + pl32(x);
    t1 = tick(x);
    if (threadIdx.x == 0) cyc[3] = t1 - t0;
    // 4: readlane + add
    t0 = tick(x);
#pragma unroll
    for (int i = 0; i < N; i++) x = x + rl(x, 3);
    t1 = tick(x);
    if (threadIdx.x == 0) cyc[4] = t1 - t0;
    // 5: independent adds (4 chains) -> throughput
    double a = x, b = x + 1, c = x + 2, d = x + 3;
    t0 = tick(x);
#pragma unroll
    for (int i = 0; i < N / 4; i++) { a = a + y; b = b + y; c = c + y; d = d + y; }
    { double z = a + b + c + d; t1 = tick(z); x = z; }
    if (threadIdx.x == 0) cyc[5] = t1 - t0;
    x = a + b + c + d;
    // 6: dependent LDS read chain (address from data)
    int idx = threadIdx.x;
    t0 = tick(x);
#pragma unroll 1
    for (int i = 0; i < N / 8; i++) { double v = lds[idx]; idx = ((int)v + i) & 63; x += v; }
    t1 = tick(x);
    if (threadIdx.x == 0) cyc[6] = (t1 - t0) * 8;
    // 7: compare + select chain
    t0 = tick(x);
#pragma unroll
    for (int i = 0; i < N; i++) x = x < y ? y : x;
    t1 = tick(x);
    if (threadIdx.x == 0) cyc[7] = t1 - t0;
    out[threadIdx.x] = x;
}
int main() {
    double* d_out; unsigned long long* d_c; double* d_y;
    hipMalloc(&d_out, 64 * 8); hipMalloc(&d_c, 16 * 8); hipMalloc(&d_y, 64 * 8);
    double hy[64];
    for (int i = 0; i < 64; i++) hy[i] = 1e-9 * (i + 1);
    hipMemcpy(d_y, hy, sizeof(hy), hipMemcpyHostToDevice);
    const char* names[] = {"add_f64", "mul_f64", "dpp+add", "permlane32+add", "readlane+add", "indep add (per op)", "lds dependent read", "cmp+select"};
    for (int rep = 0; rep < 3; rep++) {
        k<<<1, 64>>>(d_out, d_c, 1.0, d_y);
        hipDeviceSynchronize();
    }
    unsigned long long c[16];
    hipMemcpy(c, d_c, sizeof(c), hipMemcpyDeviceToHost);
    for (int i = 0; i < 8; i++) printf("%-22s %.1f cycles/step\n", names[i], (double)c[i] / N);
    // also wall-clock calibration: 2^20 dependent adds
    return 0;
}
