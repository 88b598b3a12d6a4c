// Row-update chain experiments (one wave per block, 1024 blocks): which part of a PGS row costs what.
#include "../../urgym_amd/csrc/ug_team.h"
#include <cstdio>
using namespace ugd;
#define R 16
template <int MODE>
__device__ __forceinline__ double row_math(double Js, double Ms, double rhs, double invD, double lo, double hi, double& imp, double& dv, double& res) {
    double prod = Js * dv;
    double dot;
    if (MODE == 2) dot = readlane_d(prod, 0) + readlane_d(prod, 16);
    else if (MODE == 3) { double red = reduce16(prod); dot = red; }
    else { double red = reduce16(prod); dot = readlane_d(red, 0) + readlane_d(red, 16); }
    double di = rhs - dot * invD;
    double sum = imp + di;
    bool below = sum < lo, above = sum > hi;
    double dn = below ? lo - imp : (above ? hi - imp : di);
    double in = below ? lo : (above ? hi : sum);
    dv = dv + Ms * dn;
    if (MODE != 4) { double x = dn * invD; x = x * x; res = res > x ? res : x; }
    imp = in;
    return in;
}
template <int P, int MODE>
__device__ __forceinline__ void chain(const double (&J)[R], const double (&M)[R], double (&imp)[R], double& dv, double& res, const double* rowd) {
    if constexpr (P < R) {
        double rhs, invD, lo, hi;
        if (MODE == 5) { rhs = g_sh.rs[P].rhs; invD = g_sh.rs[P].invD; lo = g_sh.rs[P].lo; hi = g_sh.rs[P].hi; }
        else { rhs = rowd[0] + P; invD = rowd[1]; lo = rowd[2]; hi = rowd[3]; }
        row_math<MODE == 5 ? 0 : MODE>(J[P], M[P], rhs, invD, lo, hi, imp[P], dv, res);
        chain<P + 1, MODE>(J, M, imp, dv, res, rowd);
    }
}
template <int MODE>
__global__ void __launch_bounds__(64, 1) k(const double* in, double* out, unsigned long long* cyc) {
    int lane = threadIdx.x;
    double J[R], M[R], imp[R];
    for (int i = lane; i < R; i += 64) { g_sh.rs[i].rhs = in[i]; g_sh.rs[i].invD = 1.0; g_sh.rs[i].lo = -1; g_sh.rs[i].hi = 1; }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < R; p++) { J[p] = in[(p * 64 + lane) % 4096] * 0.1; M[p] = J[p] * 0.01; imp[p] = 0; }
    double rowd[4] = {in[1] * 0, 1.0, -1.0, 1.0};
    double dv = 0.0, res = 0.0;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 50; it++) {
        asm volatile("" : "+v"(dv));
        chain<0, MODE>(J, M, imp, dv, res, rowd);
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    double s = dv + res;
    for (int p = 0; p < R; p++) s += imp[p];
    out[blockIdx.x * 64 + lane] = s;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int MODE>
void run(const char* name, double* d_in, double* d_out, unsigned long long* d_c) {
    for (int r = 0; r < 2; r++) { k<MODE><<<1024, 64>>>(d_in, d_out, d_c); hipDeviceSynchronize(); }
    unsigned long long c[1024];
    hipMemcpy(c, d_c, sizeof(c), hipMemcpyDeviceToHost);
    double a = 0;
    for (int i = 0; i < 1024; i++) a += c[i];
    printf("%-40s %.1f cycles/row\n", name, a / 1024 / (50.0 * R));
}
int main() {
    double *d_in, *d_out; unsigned long long* d_c;
    hipMalloc(&d_in, 4096 * 8); hipMalloc(&d_out, 1024 * 64 * 8); hipMalloc(&d_c, 1024 * 8);
    double h[4096];
    for (int i = 0; i < 4096; i++) h[i] = ((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>("full (reduce16 + readlane, reg data)", d_in, d_out, d_c);
    run<2>("no DPP (readlane of product)", d_in, d_out, d_c);
    run<3>("no readlane (dot = reduce16 lanes)", d_in, d_out, d_c);
    run<4>("full minus residual", d_in, d_out, d_c);
    run<5>("full + LDS row data", d_in, d_out, d_c);
    return 0;
}
