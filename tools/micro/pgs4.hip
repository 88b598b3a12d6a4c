// The contact-free 12-row PGS sweep (development aid): cycles per sweep of 12 rows (lanes 0..11, one slot),
// 50 sweeps alternating direction, one wave per SIMD, with the per-sweep finish (impulse advance, residual)
// and the wave-wide convergence test as in ug_team.h passes_free12:
//   0  production before the DPP change: max, min, readlane pair, fma with the SGPR delta, cndmask record
//   1  DPP: max, min, s_nop 1, v_fmac_f64_dpp row_newbcast (the broadcast inside the fma), cndmask record
//   2  as 1 without the finish and the convergence test (the rows alone)
//   3  as 1 with the convergence branch of sweep k taken after the first 4 rows of sweep k + 1 (speculative
//      rows touch only u and the records, which a converged solve does not read)
// Usage: hipcc -O3 --offload-arch=gfx950 -o pgs4 pgs4.hip && ./pgs4
#include <hip/hip_runtime.h>
#include <cstdio>
#define NR 12

__device__ __forceinline__ double readlane_d(double x, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), l), hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}
template <int L>
__device__ __forceinline__ double own_lane_sel(double old, double x) {
    return __builtin_amdgcn_inverse_ballot_w64(1ull << L) ? x : old;
}
template <int O>
__device__ __forceinline__ double clamp_fma_bcast16(double a, double dlo, double dhi, double& w) {
    double dn;
    asm("v_max_f64 %0, %1, %2\n\t"
        "v_min_f64 %0, %0, %3\n\t"
        "s_nop 1\n\t"
        "v_fmac_f64_dpp %1, %0, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
        : "=&v"(dn), "+v"(w)
        : "v"(dlo), "v"(dhi), "v"(a), "i"(O));
    return dn;
}
template <int MODE, int P, int STEP, int K>
__device__ __forceinline__ void rows(const double (&A)[NR], double dlo, double dhi, double& W, double& dsv) {
    if constexpr (K > 0) {
        if constexpr (MODE == 0) {
            double dn = __builtin_fmin(__builtin_fmax(W, dlo), dhi);
            double d = readlane_d(dn, P);
            W = __builtin_fma(A[P], d, W);
            dsv = own_lane_sel<P>(dsv, dn);
        } else {
            const double dn = clamp_fma_bcast16<P>(A[P], dlo, dhi, W);
            dsv = own_lane_sel<P>(dsv, dn);
        }
        rows<MODE, P + STEP, STEP, K - 1>(A, dlo, dhi, W, dsv);
    }
}
__device__ __forceinline__ void finish(double& dsv, double rinv, bool did, double lo, double hi, double& imp,
                                       double& dlo, double& dhi, double& res) {
    double x = dsv * rinv;
    x = x * x;
    double r2 = res > x ? res : x;
    res = did ? r2 : res;
    imp = did ? imp + dsv : imp;
    dlo = lo - imp;
    dhi = hi - imp;
}
template <int MODE>
__global__ void __launch_bounds__(64, 1) k(const double* in, double* out, unsigned long long* cyc, double thr) {
    const int lane = threadIdx.x;
    double A[NR];
#pragma unroll
    for (int p = 0; p < NR; p++) A[p] = -in[(p * 64 + lane) % 4096] * 1e-2;
    const double lo = -1.0 - in[lane], hi = 1.0 + in[lane + 1], rinv = 1.0 + in[lane + 2];
    double W = in[lane + 128], dsv = 0.0, imp = 0.0, dlo = lo, dhi = hi;
    const bool did = lane < NR;
    int iters = 0;
    unsigned long long t0 = __builtin_readcyclecounter();
    if constexpr (MODE == 3) {
        double res = 0.0;
        rows<1, NR - 1, -1, NR>(A, dlo, dhi, W, dsv);
        finish(dsv, rinv, did, lo, hi, imp, dlo, dhi, res);
        for (int it = 0;; it++) {
            iters++;
            const bool fwd = it & 1 ? false : true; /* the sweep after sweep it */
            unsigned long long conv = __ballot(!(res <= thr));
            res = 0.0;
            if (fwd) rows<1, 0, 1, 4>(A, dlo, dhi, W, dsv);
            else rows<1, NR - 1, -1, 4>(A, dlo, dhi, W, dsv);
            if (conv == 0ull || it >= 49) break;
            if (fwd) rows<1, 4, 1, NR - 4>(A, dlo, dhi, W, dsv);
            else rows<1, NR - 5, -1, NR - 4>(A, dlo, dhi, W, dsv);
            finish(dsv, rinv, did, lo, hi, imp, dlo, dhi, res);
        }
    } else {
        for (int it = 0; it < 50; it++) {
            iters++;
            double res = 0.0;
            if (!(it & 1)) rows<MODE, NR - 1, -1, NR>(A, dlo, dhi, W, dsv);
            else rows<MODE, 0, 1, NR>(A, dlo, dhi, W, dsv);
            if constexpr (MODE != 2) {
                finish(dsv, rinv, did, lo, hi, imp, dlo, dhi, res);
                if (__ballot(!(res <= thr)) == 0ull || it >= 49) break;
            } else {
                asm volatile("" : "+v"(W), "+v"(dsv));
            }
        }
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[(blockIdx.x * 64 + lane) * 3 + 0] = W;
    out[(blockIdx.x * 64 + lane) * 3 + 1] = imp;
    out[(blockIdx.x * 64 + lane) * 3 + 2] = dsv;
    if (lane == 0) cyc[blockIdx.x] = (t1 - t0) * 1000 + iters;
}
static double href[1024 * 64 * 3];
template <int MODE>
void run(const char* name, double* d_in, double* d_out, unsigned long long* d_c, int blocks, bool ref) {
    for (int r = 0; r < 2; r++) { k<MODE><<<blocks, 64>>>(d_in, d_out, d_c, -1.0); hipDeviceSynchronize(); }
    static unsigned long long c[1024];
    static double h[1024 * 64 * 3];
    hipMemcpy(c, d_c, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    double a = 0;
    int it = 0;
    for (int i = 0; i < blocks; i++) a += c[i] / 1000, it = c[i] % 1000;
    int same = 1;
    if (ref) for (int i = 0; i < blocks * 64 * 3; i++) href[i] = h[i];
    else for (int b = 0; b < blocks; b++) for (int l = 0; l < NR; l++) for (int j = 1; j < 3; j++)
        same &= h[(b * 64 + l) * 3 + j] == href[(b * 64 + l) * 3 + j];
    printf("%-64s %7.1f cycles/sweep (%d sweeps) impulses %s\n", name, a / blocks / it, it,
           ref ? "(reference)" : same ? "identical" : "DIFFER");
}
int main() {
    double *d_in, *d_out;
    unsigned long long* d_c;
    hipMalloc(&d_in, 4096 * 8); hipMalloc(&d_out, 1024 * 64 * 3 * 8); hipMalloc(&d_c, 1024 * 8);
    static double h[4096];
    for (int i = 0; i < 4096; i++) h[i] = ((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
    const int blocks = 1024;
    run<0>("0 readlane + SGPR fma, finish, convergence test", d_in, d_out, d_c, blocks, true);
    run<1>("1 DPP row_newbcast fma, finish, convergence test", d_in, d_out, d_c, blocks, false);
    run<2>("2 DPP rows only", d_in, d_out, d_c, blocks, false);
    run<3>("3 DPP, convergence branch after 4 speculative rows", d_in, d_out, d_c, blocks, false);
    return 0;
}
