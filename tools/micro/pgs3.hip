// Per-instruction cost of the PGS row update (development aid): 48 rows, one slot, 50 sweeps, one wave per
// SIMD, variants that drop or replace one part of ug_team.h row_upd at a time (results differ by design
// except where noted):
//   0  production order: max, min, readlane pair, fma, writelane pair (columns in VGPRs)
//   1  columns pinned to AGPRs (accvgpr reads on the row)
//   2  no writelane record
//   3  no min (clamp below only)
//   4  no writelane, no min
//   5  record by v_cndmask on lane == row (dsv = own dn) instead of writelane (same records as 0)
//   6  two u slots (the fma on slot 1 too), columns in VGPRs
//   7  only fma + readlane pair (the broadcast chain without clamp or record)
// Usage: hipcc -O3 --offload-arch=gfx950 -o pgs3 pgs3.hip && ./pgs3
#include <hip/hip_runtime.h>
#include <cstdio>
#define NR 48

__device__ __forceinline__ double readlane_d(double x, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), l), hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}
template <int L>
__device__ __forceinline__ double writelane_d(double old, double x) {
    int lo = __double2loint(old), hi = __double2hiint(old);
    const int xl = __builtin_amdgcn_readfirstlane(__double2loint(x)), xh = __builtin_amdgcn_readfirstlane(__double2hiint(x));
    asm("v_writelane_b32 %0, %1, %2" : "+v"(lo) : "s"(xl), "i"(L));
    asm("v_writelane_b32 %0, %1, %2" : "+v"(hi) : "s"(xh), "i"(L));
    return __hiloint2double(hi, lo);
}
template <int MODE, int P>
__device__ __forceinline__ void rows(const double (&A)[NR], const double (&A1)[NR], int lane, double lo, double hi,
                                     double& W, double& W1, double& dsv) {
    if constexpr (P < NR) {
        double dn = (MODE == 7) ? W : (MODE == 3 || MODE == 4) ? __builtin_fmax(W, lo) : __builtin_fmin(__builtin_fmax(W, lo), hi);
        double d = readlane_d(dn, P);
        W = __builtin_fma(A[P], d, W);
        if (MODE == 6) W1 = __builtin_fma(A1[P], d, W1);
        if (MODE == 5) dsv = lane == P ? dn : dsv;
        else if (MODE != 2 && MODE != 4 && MODE != 7) dsv = writelane_d<P>(dsv, d);
        rows<MODE, P + 1>(A, A1, lane, lo, hi, W, W1, dsv);
    }
}
template <int MODE>
__global__ void __launch_bounds__(64, 1) k(const double* in, double* out, unsigned long long* cyc) {
    const int lane = threadIdx.x;
    double A[NR], A1[NR];
#pragma unroll
    for (int p = 0; p < NR; p++) {
        A[p] = -in[(p * 64 + lane) % 4096] * 1e-2;
        A1[p] = MODE == 6 ? -in[(p * 64 + lane + 5) % 4096] * 1e-2 : 0.0;
    }
    if (MODE == 1) {
#pragma unroll
        for (int p = 0; p < NR; p++) asm volatile("" : "+a"(A[p]));
    }
    double lo = -1.0 - in[lane], hi = 1.0 + in[lane + 1], W = in[lane + 128], W1 = in[lane + 192], dsv = 0.0;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 50; it++) {
        rows<MODE, 0>(A, A1, lane, lo, hi, W, W1, dsv);
        asm volatile("" : "+v"(W), "+v"(W1), "+v"(dsv));
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[(blockIdx.x * 64 + lane) * 3 + 0] = W;
    out[(blockIdx.x * 64 + lane) * 3 + 1] = W1;
    out[(blockIdx.x * 64 + lane) * 3 + 2] = dsv;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int MODE>
void run(const char* name, double* d_in, double* d_out, unsigned long long* d_c, int blocks) {
    for (int r = 0; r < 2; r++) { k<MODE><<<blocks, 64>>>(d_in, d_out, d_c); hipDeviceSynchronize(); }
    static unsigned long long c[1024];
    hipMemcpy(c, d_c, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double a = 0;
    for (int i = 0; i < blocks; i++) a += c[i];
    printf("%-52s %6.1f cycles/row\n", name, a / blocks / (50.0 * NR));
}
int main() {
    double *d_in, *d_out;
    unsigned long long* d_c;
    hipMalloc(&d_in, 4096 * 8); hipMalloc(&d_out, 1024 * 64 * 3 * 8); hipMalloc(&d_c, 1024 * 8);
    static double h[4096];
    for (int i = 0; i < 4096; i++) h[i] = ((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
    const int blocks = 1024;
    run<0>("0 production (VGPR columns)", d_in, d_out, d_c, blocks);
    run<1>("1 columns in AGPRs", d_in, d_out, d_c, blocks);
    run<2>("2 no writelane record", d_in, d_out, d_c, blocks);
    run<3>("3 no min", d_in, d_out, d_c, blocks);
    run<4>("4 no min, no record", d_in, d_out, d_c, blocks);
    run<5>("5 record by cndmask on own lane", d_in, d_out, d_c, blocks);
    run<6>("6 two u slots", d_in, d_out, d_c, blocks);
    run<7>("7 fma + readlane only", d_in, d_out, d_c, blocks);
    return 0;
}
