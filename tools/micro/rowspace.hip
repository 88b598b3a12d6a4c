// Row-space PGS row-update microbenchmark (one wave per block, 1024 blocks): cycles per row of the
// team_pgs inner step (ug_team.h row_upd) with and without the per-row range branches, and variants of
// the chain (no writelane record, no slot-1 fma, clamp by compare/select).
#include "../../urgym_amd/csrc/ug_team.h"
#include <cstdio>
using namespace ugd;
#define R 64
template <int P, int MODE>
__device__ __forceinline__ void chain(const double (&A0)[PREG], const double (&A1)[PREG], int lane, int start, int end,
                                      Lrow& L, double (&W)[2]) {
    if constexpr (P < R) {
        if (MODE == 1) {
            if (P < end) {
                if (P >= start) row_upd<P>(A0, A1, nullptr, lane, L, W);
                chain<P + 1, MODE>(A0, A1, lane, start, end, L, W);
            }
        } else if (MODE == 0) {
            row_upd<P>(A0, A1, nullptr, lane, L, W);
            chain<P + 1, MODE>(A0, A1, lane, start, end, L, W);
        } else if (MODE == 2) { /* no record */
            constexpr int s = P >> 6, O = P & 63;
            double dn = __builtin_fmin(__builtin_fmax(W[s], L.dlo[s]), L.dhi[s]);
            double d = readlane_d(dn, O);
            W[0] = __builtin_fma(A0[P], d, W[0]);
            W[1] = __builtin_fma(A1[P], d, W[1]);
            chain<P + 1, MODE>(A0, A1, lane, start, end, L, W);
        } else if (MODE == 3) { /* no record, one slot */
            constexpr int O = P & 63;
            double dn = __builtin_fmin(__builtin_fmax(W[0], L.dlo[0]), L.dhi[0]);
            double d = readlane_d(dn, O);
            W[0] = __builtin_fma(A0[P], d, W[0]);
            chain<P + 1, MODE>(A0, A1, lane, start, end, L, W);
        } else if (MODE == 4) { /* readlane + fma only */
            constexpr int O = P & 63;
            double d = readlane_d(W[0], O);
            W[0] = __builtin_fma(A0[P], d, W[0]);
            chain<P + 1, MODE>(A0, A1, lane, start, end, L, W);
        } else if (MODE == 5) { /* fma chain only (no broadcast) */
            W[0] = __builtin_fma(A0[P], W[0], W[1]);
            chain<P + 1, MODE>(A0, A1, lane, start, end, L, W);
        }
    }
}
template <int MODE>
__global__ void __launch_bounds__(64, 1) k(const double* in, double* out, unsigned long long* cyc, int start, int end) {
    int lane = threadIdx.x;
    double A0[PREG], A1[PREG];
#pragma unroll
    for (int p = 0; p < PREG; p++) { A0[p] = -in[(p * 64 + lane) % 4096] * 1e-3; A1[p] = A0[p] * 0.5; }
    Lrow L;
    for (int s = 0; s < 2; s++) {
        L.dlo[s] = -1.0 - in[lane]; L.dhi[s] = 1.0 + in[lane]; L.dsv[s] = 0; L.rhs[s] = in[lane + 64];
        L.invD[s] = 1; L.rinv[s] = 1; L.lo[s] = -1; L.hi[s] = 1; L.imp[s] = 0;
    }
    double W[2] = {in[lane + 128], in[lane + 192]};
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 50; it++) {
        int s0 = start, e0 = end;
        asm volatile("" : "+s"(s0), "+s"(e0));
        chain<0, MODE>(A0, A1, lane, s0, e0, L, W);
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x * 64 + lane] = W[0] + W[1] + L.dsv[0];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int MODE>
void run(const char* name, double* d_in, double* d_out, unsigned long long* d_c, int blocks) {
    for (int r = 0; r < 2; r++) { k<MODE><<<blocks, 64>>>(d_in, d_out, d_c, 0, R); hipDeviceSynchronize(); }
    unsigned long long c[1024];
    hipMemcpy(c, d_c, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double a = 0;
    for (int i = 0; i < blocks; i++) a += c[i];
    printf("%-44s blocks %4d: %.1f cycles/row\n", name, blocks, a / blocks / (50.0 * R));
}
int main() {
    double *d_in, *d_out; unsigned long long* d_c;
    hipMalloc(&d_in, 4096 * 8); hipMalloc(&d_out, 1024 * 64 * 8); hipMalloc(&d_c, 1024 * 8);
    double h[4096];
    for (int i = 0; i < 4096; i++) h[i] = ((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int blocks : {256, 1024}) {
        run<1>("row_upd + range branches (as in team_pgs)", d_in, d_out, d_c, blocks);
        run<0>("row_upd, no branches", d_in, d_out, d_c, blocks);
        run<2>("no writelane record", d_in, d_out, d_c, blocks);
        run<3>("no record, one slot", d_in, d_out, d_c, blocks);
        run<4>("readlane pair + fma only", d_in, d_out, d_c, blocks);
        run<5>("dependent fma only", d_in, d_out, d_c, blocks);
    }
    return 0;
}
