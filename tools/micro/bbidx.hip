// Reproducer for VERDICT r2 item 7 (team_box_box read the wrong rotation column with run-time indices).
// One wave per box pair runs team_box_box's separating-axis selection (15 tests one per lane, the serial
// selection replayed on readlane broadcasts) and then forms the reference-face normal three ways:
//   dyn  const m3& Rn = nR < 3 ? R1 : R2;  Rn.m[c], Rn.m[3 + c], Rn.m[6 + c]   (the original code)
//   sel  the same column by explicit selects                                    (the shipped code)
//   host the serial selection on the CPU
// and counts the pairs where dyn or sel disagree with host.  TA / TB are locals of a __noinline__ device function
// that keeps them in its private frame (as team_collide's XF locals were).  The root cause shows in the ISA
// (python tools/scc_audit.py on the -S output): frame-index elimination materialises the second object's address
// with `s_add_i32 sX, s33, imm` -- an SCC-writing add -- between `s_and_b64 ..., vcc, exec` (SCC = nR < 3) and the
// `s_cselect_b32` that picks the base address, so the pick always takes R2.
// Usage: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o bbidx bbidx.hip && ./bbidx
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct v3 { double x, y, z; };
struct m3 { double m[9]; };
struct XF { m3 R; v3 p; };
__host__ __device__ inline v3 V(double x, double y, double z) { return v3{x, y, z}; }
__host__ __device__ inline m3 qmat(const double* q) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    m3 R;
    R.m[0] = 1 - 2 * (y * y + z * z); R.m[1] = 2 * (x * y - z * w); R.m[2] = 2 * (x * z + y * w);
    R.m[3] = 2 * (x * y + z * w); R.m[4] = 1 - 2 * (x * x + z * z); R.m[5] = 2 * (y * z - x * w);
    R.m[6] = 2 * (x * z - y * w); R.m[7] = 2 * (y * z + x * w); R.m[8] = 1 - 2 * (x * x + y * y);
    return R;
}
__host__ __device__ inline double col_dot(const m3& A, int i, const m3& B, int j) {
    return A.m[i] * B.m[j] + A.m[3 + i] * B.m[3 + j] + A.m[6 + i] * B.m[6 + j];
}
__host__ __device__ inline double col_dotv(const m3& A, int i, v3 v) { return A.m[i] * v.x + A.m[3 + i] * v.y + A.m[6 + i] * v.z; }
__device__ inline double readlane_d(double x, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), l), hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}

/* the 15 axis tests (ODE dBoxBox2): separation s2 of test t, and e1 (for the normal's sign) */
__host__ __device__ inline void axis_test(int t, const m3& R1, const m3& R2, v3 p, const double* Ah, const double* Bh,
                                          double& e1, double& x2) {
    const v3 pp = V(col_dotv(R1, 0, p), col_dotv(R1, 1, p), col_dotv(R1, 2, p));
    const double R11 = col_dot(R1, 0, R2, 0), R12 = col_dot(R1, 0, R2, 1), R13 = col_dot(R1, 0, R2, 2);
    const double R21 = col_dot(R1, 1, R2, 0), R22 = col_dot(R1, 1, R2, 1), R23 = col_dot(R1, 1, R2, 2);
    const double R31 = col_dot(R1, 2, R2, 0), R32 = col_dot(R1, 2, R2, 1), R33 = col_dot(R1, 2, R2, 2);
    const double Q11 = fabs(R11), Q12 = fabs(R12), Q13 = fabs(R13), Q21 = fabs(R21), Q22 = fabs(R22), Q23 = fabs(R23);
    const double Q31 = fabs(R31), Q32 = fabs(R32), Q33 = fabs(R33);
    e1 = 0.0; x2 = 0.0;
    switch (t) {
    case 0: e1 = pp.x; x2 = (Ah[0] + Bh[0] * Q11 + Bh[1] * Q12 + Bh[2] * Q13); break;
    case 1: e1 = pp.y; x2 = (Ah[1] + Bh[0] * Q21 + Bh[1] * Q22 + Bh[2] * Q23); break;
    case 2: e1 = pp.z; x2 = (Ah[2] + Bh[0] * Q31 + Bh[1] * Q32 + Bh[2] * Q33); break;
    case 3: e1 = col_dotv(R2, 0, p); x2 = (Ah[0] * Q11 + Ah[1] * Q21 + Ah[2] * Q31 + Bh[0]); break;
    case 4: e1 = col_dotv(R2, 1, p); x2 = (Ah[0] * Q12 + Ah[1] * Q22 + Ah[2] * Q32 + Bh[1]); break;
    case 5: e1 = col_dotv(R2, 2, p); x2 = (Ah[0] * Q13 + Ah[1] * Q23 + Ah[2] * Q33 + Bh[2]); break;
    default: break;
    }
}

__device__ __noinline__ void escape(XF* a, XF* b) { asm volatile("" : : "v"(a), "v"(b) : "memory"); }

template <bool DYN>
__device__ __forceinline__ v3 face_normal(const XF& TA, const XF& TB, const double (&Ah)[3], const double (&Bh)[3],
                                          int& nR_out) {
    const int lane = threadIdx.x;
    const m3& R1 = TA.R;
    const m3& R2 = TB.R;
    const v3 p = V(TB.p.x - TA.p.x, TB.p.y - TA.p.y, TB.p.z - TA.p.z);
    double e1, x2;
    axis_test(lane < 6 ? lane : 15, R1, R2, p, Ah, Bh, e1, x2);
    const double s2 = fabs(e1) - x2;
    double s = -1e300;
    int nR = -1;
    for (int t = 0; t < 6; t++) {
        const double v = readlane_d(s2, t);
        if (v > s) { s = v; nR = t; }
    }
    nR_out = nR;
    v3 normal = V(0, 0, 0);
    if (nR >= 0) {
        const m3& Rn = nR < 3 ? R1 : R2;
        const int c = nR % 3;
        if (DYN) normal = V(Rn.m[c], Rn.m[3 + c], Rn.m[6 + c]);
        else normal = c == 0 ? V(Rn.m[0], Rn.m[3], Rn.m[6]) : c == 1 ? V(Rn.m[1], Rn.m[4], Rn.m[7]) : V(Rn.m[2], Rn.m[5], Rn.m[8]);
    }
    return normal;
}

__device__ __noinline__ void pick_both(const double* q, double* o, int* nr) {
    XF TA, TB;
    TA.R = qmat(q); TA.p = V(q[4], q[5], q[6]);
    TB.R = qmat(q + 7); TB.p = V(q[11], q[12], q[13]);
    escape(&TA, &TB); /* keep both objects in this function's private frame, as team_collide's XF locals were */
    const double Ah[3] = {0.02, 0.02, 0.02}, Bh[3] = {0.02, 0.02, 0.02};
    int n0, n1;
    const v3 a = face_normal<true>(TA, TB, Ah, Bh, n0);
    const v3 b = face_normal<false>(TA, TB, Ah, Bh, n1);
    if (threadIdx.x == 0) {
        o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = b.x; o[4] = b.y; o[5] = b.z;
        *nr = n0;
    }
}
__global__ void __launch_bounds__(64) k_pick(const double* in, double* out, int* nr) {
    pick_both(in + 14 * blockIdx.x, out + 6 * blockIdx.x, nr + blockIdx.x);
}

static void rq(double* q) {
    double n = 0;
    for (int i = 0; i < 4; i++) { q[i] = rand() / (double)RAND_MAX - 0.5; n += q[i] * q[i]; }
    n = sqrt(n);
    for (int i = 0; i < 4; i++) q[i] /= n;
}

int main() {
    const int N = 4096;
    std::vector<double> in(14 * N), out(6 * N);
    std::vector<int> nr(N);
    srand(7);
    for (int i = 0; i < N; i++) {
        double* q = &in[14 * i];
        if (i & 1) { q[0] = q[1] = q[2] = 0.0; q[3] = 1.0; } else rq(q);
        q[4] = 0.1; q[5] = -0.6; q[6] = 0.02;
        rq(q + 7);
        q[11] = 0.1 + 0.01 * (rand() / (double)RAND_MAX - 0.5); q[12] = -0.6; q[13] = 0.02 + 0.035 + 0.01 * (rand() / (double)RAND_MAX);
    }
    double *din, *dout;
    int* dnr;
    hipMalloc(&din, sizeof(double) * in.size());
    hipMalloc(&dout, sizeof(double) * out.size());
    hipMalloc(&dnr, sizeof(int) * N);
    hipMemcpy(din, in.data(), sizeof(double) * in.size(), hipMemcpyHostToDevice);
    k_pick<<<N, 64>>>(din, dout, dnr);
    hipMemcpy(out.data(), dout, sizeof(double) * out.size(), hipMemcpyDeviceToHost);
    hipMemcpy(nr.data(), dnr, sizeof(int) * N, hipMemcpyDeviceToHost);
    int bad_dyn = 0, bad_sel = 0, shown = 0;
    for (int i = 0; i < N; i++) {
        const double* q = &in[14 * i];
        m3 R1 = qmat(q), R2 = qmat(q + 7);
        v3 p = V(q[11] - q[4], q[12] - q[5], q[13] - q[6]);
        const double Ah[3] = {0.02, 0.02, 0.02}, Bh[3] = {0.02, 0.02, 0.02};
        double s = -1e300;
        int n = -1;
        for (int t = 0; t < 6; t++) {
            double e1, x2;
            axis_test(t, R1, R2, p, Ah, Bh, e1, x2);
            const double v = fabs(e1) - x2;
            if (v > s) { s = v; n = t; }
        }
        const m3& Rn = n < 3 ? R1 : R2;
        const int c = n % 3;
        const double h[3] = {Rn.m[c], Rn.m[3 + c], Rn.m[6 + c]};
        const double* o = &out[6 * i];
        const bool bd = o[0] != h[0] || o[1] != h[1] || o[2] != h[2];
        const bool bs = o[3] != h[0] || o[4] != h[1] || o[5] != h[2];
        bad_dyn += bd;
        bad_sel += bs;
        if ((bd || bs) && shown < 4) {
            printf("pair %d nR host %d gpu %d  host (%.6f %.6f %.6f) dyn (%.6f %.6f %.6f) sel (%.6f %.6f %.6f)\n", i, n, nr[i],
                   h[0], h[1], h[2], o[0], o[1], o[2], o[3], o[4], o[5]);
            shown++;
        }
    }
    printf("pairs %d: dyn mismatches %d, sel mismatches %d\n", N, bad_dyn, bad_sel);
    return 0;
}
