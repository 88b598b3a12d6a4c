// Check of the MFMA Delassus build used by team_pgs: 4 row tiles x 16-column block of
// A[i][p] = fma-chain_d J_i[d] * MJ_p[d] (K = 24) via v_mfma_f64_16x16x4_f64, then a 4x4 lane-row/register
// transpose (permlane32_swap, permlane16_swap) so that lane l holds A[l][16 pb + c], c = 0..15.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void swap32(double& x, double& y) {
    unsigned xl = __double2loint(x), xh = __double2hiint(x), yl = __double2loint(y), yh = __double2hiint(y);
    auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    x = __hiloint2double(h[0], l[0]);
    y = __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ void swap16(double& x, double& y) {
    unsigned xl = __double2loint(x), xh = __double2hiint(x), yl = __double2loint(y), yh = __double2hiint(y);
    auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
    auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
    x = __hiloint2double(h[0], l[0]);
    y = __hiloint2double(h[1], l[1]);
}
// J: 64 rows x 24, MJ: 16 rows (columns p) x 24; out[l*16 + c] = A[l][c]; ref computed per lane
__global__ void k(const double* J, const double* MJ, double* out, double* ref) {
    const int l = threadIdx.x;
    d4 acc[4];
    for (int g = 0; g < 4; g++) acc[g] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 6; ks++) {
        double a = MJ[(l & 15) * 24 + 4 * ks + (l >> 4)];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            double b = J[(16 * g + (l & 15)) * 24 + 4 * ks + (l >> 4)];
            acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[g], 0, 0, 0);
        }
    }
    double W[4][4]; // [h][r]
#pragma unroll
    for (int r = 0; r < 4; r++) {
        double v0 = acc[0][r], v1 = acc[1][r], v2 = acc[2][r], v3 = acc[3][r];
        swap32(v0, v2);
        swap32(v1, v3);
        swap16(v0, v1);
        swap16(v2, v3);
        W[0][r] = v0; W[1][r] = v1; W[2][r] = v2; W[3][r] = v3;
    }
    for (int h = 0; h < 4; h++)
        for (int r = 0; r < 4; r++) out[l * 16 + h + 4 * r] = W[h][r];
    for (int c = 0; c < 16; c++) {
        double s = 0.0;
        for (int d = 0; d < 24; d++) s = __builtin_fma(J[l * 24 + d], MJ[c * 24 + d], s);
        ref[l * 16 + c] = s;
    }
}
int main() {
    double *J, *MJ, *O, *R;
    hipMallocManaged(&J, 64 * 24 * 8); hipMallocManaged(&MJ, 16 * 24 * 8);
    hipMallocManaged(&O, 64 * 16 * 8); hipMallocManaged(&R, 64 * 16 * 8);
    srand(3);
    long bad = 0, tot = 0;
    for (int trial = 0; trial < 100; trial++) {
        for (int i = 0; i < 64 * 24; i++) J[i] = ((double)rand() / RAND_MAX - 0.5) * pow(10.0, rand() % 8 - 4);
        for (int i = 0; i < 16 * 24; i++) MJ[i] = ((double)rand() / RAND_MAX - 0.5) * pow(10.0, rand() % 8 - 4);
        k<<<1, 64>>>(J, MJ, O, R);
        hipDeviceSynchronize();
        for (int e = 0; e < 64 * 16; e++) { tot++; bad += O[e] != R[e]; }
    }
    printf("MFMA build + permlane transpose vs per-lane fma chain: %ld / %ld differ\n", bad, tot);
    return 0;
}
