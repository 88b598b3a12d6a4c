// Row-space PGS sweep microbenchmark, in-situ conditions (development aid): 74 rows (slot 1 present), the
// 2 x PREG Delassus register columns (so the compiler spills part of them to AGPRs as in team_pgs), 50 sweeps.
// Variants (all must produce bit-identical u / records):
//   0  ug_team.h row_upd as used by team_pgs (clamp, readlane broadcast, fma per slot, writelane record)
//   1  software-pipelined row_upd: next row's column read ahead, the critical slot's fma first
//   2  chunk-redundant chain: per 8-row chunk every lane runs the chunk's Gauss-Seidel chain on uniform copies
//      (u by readlane at chunk start, bounds and the chunk's lower-triangular block of the Delassus matrix
//      broadcast from LDS), then the bulk fma updates of its own rows (same operands, same order)
//   3  variant 0 with the slot-1 columns pinned to AGPRs by an "a" asm constraint (A0 in VGPRs)
//   4  the production section structure (ug_team.h sweep_section): non-contact rows [0, 12) reversed on even
//      sweeps, then [12 | 0, 33), then [33, 74), each section over whole CHUNK-row chunks with neutral rows
//      (same row count per sweep as BallBalance in situ; records differ from variant 0 by design)
//   5  one chunked section over all 74 rows (the chunk tests alone)
//   7  variant 0 with an opaque always-true scalar test around every 8 rows (the cost of one chunk test)
//   8  the same with one test per 16 rows
//   9  variant 4 with an 80-position span (10 chunk positions per section instead of 16)
//   6  variant 4 with switch dispatch: a jump into the section's first chunk, one exit compare per chunk
//      (must equal variant 4 bit for bit)
// Usage: tools/micro/pgs2 (prints cycles per row update and a bit-exactness check against variant 0)
#include "../../urgym_amd/csrc/ug_team.h"
#include <cstdio>
#include <cstring>
using namespace ugd;
#define NR 74
#define NCH ((NR + 7) / 8)

template <int P>
__device__ __forceinline__ void colv(const double (&A0)[PREG], const double (&A1)[PREG], double& a0, double& a1) {
    a0 = A0[P < PREG ? P : 0];
    a1 = A1[P < PREG ? P : 0];
}
/* variant 0: the production row update */
template <int P>
__device__ __forceinline__ void v0_rows(const double (&A0)[PREG], const double (&A1)[PREG], int lane, Lrow& L,
                                        double (&W)[2]) {
    if constexpr (P < NR) {
        row_upd<P, true>(A0, A1, nullptr, lane, L, W);
        v0_rows<P + 1>(A0, A1, lane, L, W);
    }
}
template <int P, int K>
__device__ __forceinline__ void v0_rows_n(const double (&A0)[PREG], const double (&A1)[PREG], int lane, Lrow& L,
                                          double (&W)[2]) {
    if constexpr (K > 0 && P < NR) {
        row_upd<P, true>(A0, A1, nullptr, lane, L, W);
        v0_rows_n<P + 1, K - 1>(A0, A1, lane, L, W);
    }
}
/* variants 7 / 8: variant 0 with an opaque always-true test around every G rows */
template <int P, int G>
__device__ __forceinline__ void vg_rows(const double (&A0)[PREG], const double (&A1)[PREG], int lane, Lrow& L,
                                        double (&W)[2], int on) {
    if constexpr (P < NR) {
        if (on > P) v0_rows_n<P, G>(A0, A1, lane, L, W);
        vg_rows<P + G, G>(A0, A1, lane, L, W, on);
    }
}
/* variant 1: column of the next row in VGPRs before this row's clamp; critical slot first */
template <int P>
__device__ __forceinline__ void v1_rows(const double (&A0)[PREG], const double (&A1)[PREG], int lane, Lrow& L,
                                        double (&W)[2], double a0, double a1) {
    if constexpr (P < NR) {
        constexpr int s = P >> 6, O = P & 63;
        double n0 = 0.0, n1 = 0.0;
        if constexpr (P + 1 < NR) colv<P + 1>(A0, A1, n0, n1);
        asm volatile("" : "+v"(n0), "+v"(n1));
        double dn = __builtin_fmin(__builtin_fmax(W[s], L.dlo[s]), L.dhi[s]);
        double d = readlane_d(dn, O);
        constexpr int sn = (P + 1) >> 6; /* slot of the next row: its fma is on the chain */
        if constexpr (sn == 0) {
            W[0] = __builtin_fma(a0, d, W[0]);
            asm volatile("" : "+v"(W[0]));
            W[1] = __builtin_fma(a1, d, W[1]);
        } else {
            W[1] = __builtin_fma(a1, d, W[1]);
            asm volatile("" : "+v"(W[1]));
            W[0] = __builtin_fma(a0, d, W[0]);
        }
        L.dsv[s] = writelane_d<O>(L.dsv[s], d);
        v1_rows<P + 1>(A0, A1, lane, L, W, n0, n1);
    }
}
/* variant 2: chunk-redundant chain */
template <int P0, int R>
__device__ __forceinline__ void v2_bulk(const double (&A0)[PREG], const double (&A1)[PREG], int lane, Lrow& L,
                                        double (&W)[2], const double (&d)[8]) {
    if constexpr (R < 8) {
        constexpr int P = P0 + R;
        double a0 = 0.0, a1 = 0.0;
        if constexpr (P < NR) colv<P>(A0, A1, a0, a1);
        W[0] = __builtin_fma(a0, d[R], W[0]);
        W[1] = __builtin_fma(a1, d[R], W[1]);
        constexpr int s = P >> 6, O = P & 63;
        if constexpr (s == 0) L.dsv[0] = lane == O ? d[R] : L.dsv[0];
        else L.dsv[1] = lane == O ? d[R] : L.dsv[1];
        v2_bulk<P0, R + 1>(A0, A1, lane, L, W, d);
    }
}
template <int C>
__device__ __forceinline__ void v2_chunks(const double (&A0)[PREG], const double (&A1)[PREG], int lane, Lrow& L,
                                          double (&W)[2], const double* tri, const double* bnd) {
    if constexpr (8 * C < NR) {
        constexpr int P0 = 8 * C;
        double u[8], d[8], lo[8], hi[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            lo[j] = bnd[2 * (P0 + j)];
            hi[j] = bnd[2 * (P0 + j) + 1];
        }
#pragma unroll
        for (int j = 0; j < 8; j++) u[j] = readlane_d(W[(P0 + j) >> 6], (P0 + j) & 63);
#pragma unroll
        for (int r = 0; r < 8; r++) {
            d[r] = __builtin_fmin(__builtin_fmax(u[r], lo[r]), hi[r]);
#pragma unroll
            for (int j = r + 1; j < 8; j++) u[j] = __builtin_fma(tri[64 * C + 8 * j + r], d[r], u[j]);
        }
        v2_bulk<P0, 0>(A0, A1, lane, L, W, d);
        v2_chunks<C + 1>(A0, A1, lane, L, W, tri, bnd);
    }
}

/* chunk sequence [c_lo, c_hi] by a jump into the first chunk and one exit compare per chunk */
#define SW_FWD(C) \
    case C: \
        chunk_rows<C, false, 0, true>(A0, A1, nullptr, lane, F, W); \
        if (c_hi == C) break; \
        [[fallthrough]];
#define SW_REV(C) \
    case C: \
        chunk_rows<C, true, 0, true>(A0, A1, nullptr, lane, F, W); \
        if (c_lo == C) break; \
        [[fallthrough]];
template <bool REV>
__device__ __forceinline__ void sweep_section_sw(const double (&A0)[PREG], const double (&A1)[PREG], int lane, int a,
                                                 int b, Lrow& L, double (&W)[2]) {
    Lrow F = L;
    bool in[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const int p = lane + 64 * s;
        in[s] = p >= a && p < b;
        F.dlo[s] = in[s] ? L.dlo[s] : 0.0;
        F.dhi[s] = in[s] ? L.dhi[s] : 0.0;
    }
    const int c_lo = a / CHUNK, c_hi = (b - 1) / CHUNK;
    if (REV) {
        switch (c_hi) { SW_REV(15) SW_REV(14) SW_REV(13) SW_REV(12) SW_REV(11) SW_REV(10) SW_REV(9) SW_REV(8)
                        SW_REV(7) SW_REV(6) SW_REV(5) SW_REV(4) SW_REV(3) SW_REV(2) SW_REV(1) SW_REV(0) default: break; }
    } else {
        switch (c_lo) { SW_FWD(0) SW_FWD(1) SW_FWD(2) SW_FWD(3) SW_FWD(4) SW_FWD(5) SW_FWD(6) SW_FWD(7) SW_FWD(8)
                        SW_FWD(9) SW_FWD(10) SW_FWD(11) SW_FWD(12) SW_FWD(13) SW_FWD(14) SW_FWD(15) default: break; }
    }
#pragma unroll
    for (int s = 0; s < 2; s++) L.dsv[s] = in[s] ? F.dsv[s] : L.dsv[s];
}

template <int MODE>
__global__ void __launch_bounds__(64, 1) k(const double* in, double* out, unsigned long long* cyc) {
    __shared__ double tri[NCH * 64];
    __shared__ double bnd[2 * NCH * 8];
    const int lane = threadIdx.x;
    double A0[PREG], A1[PREG];
#pragma unroll
    for (int p = 0; p < PREG; p++) {
        A0[p] = p < NR ? -in[(p * 64 + lane) % 4096] * 1e-2 : 0.0;
        A1[p] = (p < NR && lane + 64 < NR) ? -in[(p * 64 + lane + 7) % 4096] * 1e-2 : 0.0;
    }
    Lrow L;
    for (int s = 0; s < 2; s++) {
        const bool in_ = lane + 64 * s < NR;
        L.dlo[s] = in_ ? -1.0 - in[lane] : 0.0; L.dhi[s] = in_ ? 1.0 + in[lane + 1] : 0.0; L.dsv[s] = 0;
        L.rhs[s] = in[lane + 64]; L.invD[s] = 1; L.rinv[s] = 1; L.lo[s] = -1; L.hi[s] = 1; L.imp[s] = 0;
    }
    double W[2] = {in[lane + 128], lane + 64 < NR ? in[lane + 192] : 0.0};
    if (MODE == 2) { /* LDS: bounds of every row, lower triangle of each chunk's diagonal block */
        for (int s = 0; s < 2; s++)
            if (lane + 64 * s < 8 * NCH) { bnd[2 * (lane + 64 * s)] = L.dlo[s]; bnd[2 * (lane + 64 * s) + 1] = L.dhi[s]; }
#pragma unroll
        for (int p = 0; p < PREG; p++) {
            if (p >= 8 * NCH) break;
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int row = lane + 64 * s;
                if ((row >> 3) == (p >> 3) && row > p) tri[64 * (p >> 3) + 8 * (row & 7) + (p & 7)] = s ? A1[p] : A0[p];
            }
        }
        __syncthreads();
    }
    if (MODE == 3) { /* slot-1 columns pinned to AGPRs (A0 stays in VGPRs) */
#pragma unroll
        for (int p = 0; p < PREG; p++) asm volatile("" : "+a"(A1[p]));
    }
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 50; it++) {
        if (MODE == 0 || MODE == 3) v0_rows<0>(A0, A1, lane, L, W);
        if (MODE == 1) { double a0, a1; colv<0>(A0, A1, a0, a1); v1_rows<0>(A0, A1, lane, L, W, a0, a1); }
        if (MODE == 2) v2_chunks<0>(A0, A1, lane, L, W, tri, bnd);
        if (MODE == 4) {
            int nnc = 12, fb = 33, n = NR;
            asm volatile("" : "+s"(nnc), "+s"(fb), "+s"(n));
            if (!(it & 1)) sweep_section<true, (NCMAX + CHUNK - 1) / CHUNK, true>(A0, A1, nullptr, lane, 0, nnc, 0ull, 0ull, L, W);
            sweep_section<false, MAXROWS / CHUNK, true>(A0, A1, nullptr, lane, (it & 1) ? 0 : nnc, fb, 0ull, 0ull, L, W);
            sweep_section<false, MAXROWS / CHUNK, true>(A0, A1, nullptr, lane, fb, n, 0ull, 0ull, L, W);
        }
        if (MODE == 7 || MODE == 8) {
            int on = 1000;
            asm volatile("" : "+s"(on));
            vg_rows<0, MODE == 7 ? 8 : 16>(A0, A1, lane, L, W, on);
        }
        if (MODE == 9) {
            int nnc = 12, fb = 33, n = NR;
            asm volatile("" : "+s"(nnc), "+s"(fb), "+s"(n));
            if (!(it & 1)) sweep_section<true, (NCMAX + CHUNK - 1) / CHUNK, true>(A0, A1, nullptr, lane, 0, nnc, 0ull, 0ull, L, W);
            sweep_section<false, 80 / CHUNK, true>(A0, A1, nullptr, lane, (it & 1) ? 0 : nnc, fb, 0ull, 0ull, L, W);
            sweep_section<false, 80 / CHUNK, true>(A0, A1, nullptr, lane, fb, n, 0ull, 0ull, L, W);
        }
        if (MODE == 5) {
            int n = NR;
            asm volatile("" : "+s"(n));
            sweep_section<false, MAXROWS / CHUNK, true>(A0, A1, nullptr, lane, 0, n, 0ull, 0ull, L, W);
        }
        if (MODE == 6) {
            int nnc = 12, fb = 33, n = NR;
            asm volatile("" : "+s"(nnc), "+s"(fb), "+s"(n));
            if (!(it & 1)) sweep_section_sw<true>(A0, A1, lane, 0, nnc, L, W);
            sweep_section_sw<false>(A0, A1, lane, (it & 1) ? 0 : nnc, fb, L, W);
            sweep_section_sw<false>(A0, A1, lane, fb, n, L, W);
        }
        asm volatile("" : "+v"(W[0]), "+v"(W[1]));
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[(blockIdx.x * 64 + lane) * 4 + 0] = W[0];
    out[(blockIdx.x * 64 + lane) * 4 + 1] = W[1];
    out[(blockIdx.x * 64 + lane) * 4 + 2] = L.dsv[0];
    out[(blockIdx.x * 64 + lane) * 4 + 3] = L.dsv[1];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int MODE>
void run(const char* name, double* d_in, double* d_out, unsigned long long* d_c, int blocks, double* ref,
         double slots = NR) {
    for (int r = 0; r < 2; r++) { k<MODE><<<blocks, 64>>>(d_in, d_out, d_c); hipDeviceSynchronize(); }
    static unsigned long long c[1024];
    static double o[1024 * 64 * 4];
    hipMemcpy(c, d_c, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    hipMemcpy(o, d_out, sizeof(double) * blocks * 64 * 4, hipMemcpyDeviceToHost);
    double a = 0;
    for (int i = 0; i < blocks; i++) a += c[i];
    int same = ref ? memcmp(o, ref, sizeof(double) * blocks * 64 * 4) == 0 : 1;
    if (!ref) memcpy(ref = o, o, 0);
    printf("%-46s blocks %4d: %6.1f cycles/row slot  %s\n", name, blocks, a / blocks / (50.0 * slots),
           ref ? (same ? "bit-exact vs variant 0" : "MISMATCH vs variant 0") : "");
}
int main() {
    double *d_in, *d_out;
    unsigned long long* d_c;
    hipMalloc(&d_in, 4096 * 8); hipMalloc(&d_out, 1024 * 64 * 4 * 8); hipMalloc(&d_c, 1024 * 8);
    static double h[4096], ref[1024 * 64 * 4];
    for (int i = 0; i < 4096; i++) h[i] = ((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
    const int blocks = 1024;
    k<0><<<blocks, 64>>>(d_in, d_out, d_c);
    hipDeviceSynchronize();
    hipMemcpy(ref, d_out, sizeof(double) * blocks * 64 * 4, hipMemcpyDeviceToHost);
    run<0>("0 production row_upd", d_in, d_out, d_c, blocks, ref);
    run<1>("1 pipelined column + critical slot first", d_in, d_out, d_c, blocks, ref);
    run<2>("2 chunk-redundant chain (LDS bounds/triangle)", d_in, d_out, d_c, blocks, ref);
    run<3>("3 production row_upd, slot-1 columns in AGPRs", d_in, d_out, d_c, blocks, ref);
    run<7>("7 variant 0 + a test per 8 rows", d_in, d_out, d_c, blocks, ref);
    run<8>("8 variant 0 + a test per 16 rows", d_in, d_out, d_c, blocks, ref);
    run<5>("5 one chunked section [0, 74)", d_in, d_out, d_c, blocks, ref, 80);
    static double ref4[1024 * 64 * 4];
    k<4><<<blocks, 64>>>(d_in, d_out, d_c);
    hipDeviceSynchronize();
    hipMemcpy(ref4, d_out, sizeof(double) * blocks * 64 * 4, hipMemcpyDeviceToHost);
    run<4>("4 production sections (92 slots/sweep avg)", d_in, d_out, d_c, blocks, ref4, 92);
    run<6>("6 sections, switch dispatch (vs variant 4)", d_in, d_out, d_c, blocks, ref4, 92);
    run<9>("9 sections, 80-position span (vs variant 4)", d_in, d_out, d_c, blocks, ref4, 92);
    return 0;
}
