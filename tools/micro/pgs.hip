// PGS-only microbenchmark: the product's team_pgs() on synthetic rows (n rows: nnc non-contact,
// nn normals, 2*nn frictions), one wavefront per env, 1024 envs; reports cycles per row update.
#include "../../urgym_amd/csrc/ug_team.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace ugd;

__global__ void __launch_bounds__(64, 1) k_pgs(double* ws_all, const RowS* rs_in, int n, int nnc, int nn, double* out,
                                               unsigned long long* cyc) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x, d = lane & 31;
    double* ws = ws_all + (size_t)blockIdx.x * WS_DOUBLES;
    for (int i = lane; i < n; i += 64) sh.rs[i] = rs_in[i];
    if (lane < 16) sh.prof[lane] = 0;
    __syncthreads();
    double RJ[NSLOT], RM[NSLOT];
#pragma unroll
    for (int sl = 0; sl < NSLOT; sl++) { RJ[sl] = 0.0; RM[sl] = 0.0; }
    load_slots<0>(ws, RJ, RM, n, d);
    unsigned long long t0 = __builtin_readcyclecounter();
    double dv, dvs;
    int split = team_pgs(ws, n, nnc, nn, d, RJ, RM, dv, dvs);
    __syncthreads();
    unsigned long long t1 = __builtin_readcyclecounter();
    out[(size_t)blockIdx.x * 64 + lane] = dv + dvs + split;
    if (lane == 0) { cyc[2 * blockIdx.x] = t1 - t0; cyc[2 * blockIdx.x + 1] = sh.prof[PC_ITERS]; }
}

int main(int argc, char** argv) {
    int n = argc > 1 ? atoi(argv[1]) : 74, nnc = argc > 2 ? atoi(argv[2]) : 14;
    int nn = (n - nnc) / 3;
    n = nnc + 3 * nn;
    const int E = 1024;
    srand(1);
    auto U = [](double a, double b) { return a + (b - a) * (rand() / (double)RAND_MAX); };
    std::vector<RowS> rs(n);
    for (int p = 0; p < n; p++) {
        RowS& r = rs[p];
        r.invD = U(0.5, 2.0); r.rinv = 1.0 / r.invD; r.rhs = U(-1, 1); r.rhsPen = 0.0; r.imp = 0.0; r.impPen = 0.0;
        r.fric = 0.5; r.kind = p < nnc ? 1 : (p < nnc + nn ? 3 : 4); r.a = 0; r.b = 0; r.nrow = 0;
        if (p < nnc) { r.lo = -0.5; r.hi = 0.5; } else { r.lo = 0.0; r.hi = 1e10; }
        if (p >= nnc && p < nnc + nn) r.rhs = U(0.1, 1.0);
    }
    std::vector<double> ws((size_t)E * WS_DOUBLES, 0.0);
    for (int e = 0; e < E; e++)
        for (int p = 0; p < n; p++)
            for (int i = 0; i < 24; i++) {
                double j = U(-0.3, 0.3);
                ws[(size_t)e * WS_DOUBLES + WS_ROWS + p * 48 + i] = j;
                ws[(size_t)e * WS_DOUBLES + WS_ROWS + p * 48 + 24 + i] = 0.05 * j;
            }
    double *d_ws, *d_out; RowS* d_rs; unsigned long long* d_c;
    hipMalloc(&d_ws, ws.size() * 8); hipMalloc(&d_out, E * 64 * 8); hipMalloc(&d_rs, n * sizeof(RowS)); hipMalloc(&d_c, E * 16);
    hipMemcpy(d_ws, ws.data(), ws.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(d_rs, rs.data(), n * sizeof(RowS), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) { k_pgs<<<E, 64>>>(d_ws, d_rs, n, nnc, nn, d_out, d_c); hipDeviceSynchronize(); }
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a); k_pgs<<<E, 64>>>(d_ws, d_rs, n, nnc, nn, d_out, d_c); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> c(2 * E);
    hipMemcpy(c.data(), d_c, E * 16, hipMemcpyDeviceToHost);
    double cy = 0, it = 0;
    for (int e = 0; e < E; e++) { cy += c[2 * e]; it += c[2 * e + 1]; }
    cy /= E; it /= E;
    printf("n=%d nnc=%d nn=%d iters=%.1f cycles=%.0f cycles/row-update=%.1f kernel_ms=%.3f\n", n, nnc, nn, it, cy, cy / (it * n), ms);
    return 0;
}
