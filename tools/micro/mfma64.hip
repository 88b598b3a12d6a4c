// Numerics check of v_mfma_f64_16x16x4_f64 (gfx950): is a K=24 product chained over 6 MFMAs bit-identical
// to the sequential fma chain  s = 0; for k in 0..23: s = fma(x[k], y[k], s)  (the oracle's rdot)?
// Also checks the C/D lane map col = lane&15, row = (lane>>4) + 4*reg.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* X, const double* Y, double* D, double* R) {
    // X: 16 rows x 24 k (row-major), Y: 24 k x 16 cols; D[row][col] via MFMA, R via VALU fma chain
    const int l = threadIdx.x;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int ks = 0; ks < 6; ks++) {
        double a = X[(l & 15) * 24 + 4 * ks + (l >> 4)];
        double b = Y[(4 * ks + (l >> 4)) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; r++) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
    for (int e = l; e < 256; e += 64) {
        int i = e / 16, j = e % 16;
        double s = 0.0;
        for (int kk = 0; kk < 24; kk++) s = __builtin_fma(X[i * 24 + kk], Y[kk * 16 + j], s);
        R[e] = s;
    }
}
int main() {
    double *X, *Y, *D, *R;
    hipMallocManaged(&X, 16 * 24 * 8); hipMallocManaged(&Y, 24 * 16 * 8);
    hipMallocManaged(&D, 256 * 8); hipMallocManaged(&R, 256 * 8);
    srand(1);
    long bad = 0, tot = 0, badmap = 0;
    for (int trial = 0; trial < 200; trial++) {
        for (int i = 0; i < 16 * 24; i++) {
            double u = (double)rand() / RAND_MAX - 0.5, v = (double)rand() / RAND_MAX;
            X[i] = u * pow(10.0, (int)(v * 12) - 6);
            if (rand() % 5 == 0) X[i] = 0.0;
        }
        for (int i = 0; i < 24 * 16; i++) {
            double u = (double)rand() / RAND_MAX - 0.5, v = (double)rand() / RAND_MAX;
            Y[i] = u * pow(10.0, (int)(v * 12) - 6);
        }
        k<<<1, 64>>>(X, Y, D, R);
        hipDeviceSynchronize();
        for (int e = 0; e < 256; e++) {
            tot++;
            if (D[e] != R[e]) {
                bad++;
                if (fabs(D[e] - R[e]) > 1e-6 * (fabs(R[e]) + 1e-300)) badmap++;
            }
        }
    }
    printf("mfma_f64_16x16x4 chained K=24 vs sequential fma chain: %ld / %ld differ (%ld beyond 1e-6 rel: map errors)\n",
           bad, tot, badmap);
    return 0;
}
