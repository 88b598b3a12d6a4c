/* gjk_host.cpp -- the kernels' convex-convex narrowphase (urgym_amd/csrc/ug_gjk.h) built for the host.
 *
 * TEST INFRASTRUCTURE: tests/test_gjk.py runs this build and the oracle's independent restatement
 * (oracle/ug_gjk_ref.h) on the same shapes and poses and asserts bit-identical results, so arithmetic-order slips in
 * the kernel header show up on the CPU before a GPU run.  The only piece that differs from the kernels is the hull
 * support query: serial here (btVector3::maxDot's first maximum over the hull, or over the direction cell's candidate
 * list for a hull with a support-cell table -- the same tables and classification as the kernels), a lane-group
 * arg-max with the same tie rule there.  The oracle always scans the whole hull, so the bit-exact comparison in
 * tests/test_gjk.py also checks the tables; tests/test_supcells.py checks them directly (ugk_host_support).
 * Built by oracle/Makefile into oracle/_build/libgjk_host.so; never linked into the product.
 */
#define UGK_FN static inline
#ifdef UG_ROBOT_R140
#include "../urgym_amd/csrc/model_data_r140.h"
#else
#include "../urgym_amd/csrc/model_data.h"
#endif
#ifdef UG_ROBOT_R140
#include "../urgym_amd/csrc/supcell_data_r140.h"
#else
#include "../urgym_amd/csrc/supcell_data.h"
#endif
#include "../urgym_amd/csrc/ug_gjk.h"
#include "../urgym_amd/csrc/ug_supcell.h"

/* the first maximum of the dot products over the candidates (vertex indices into the hull, ascending) */
static int scan_first_max(int v0, const int* cand, int n, ugk::gv d) {
    double best = -__builtin_inf();
    int bi = 0;
    for (int k = 0; k < n; k++) {
        const int i = cand ? cand[k] : k;
        const double* p = &UG_HULL_V[3 * (v0 + i)];
        const double dd = p[0] * d.x + p[1] * d.y + p[2] * d.z;
        if (dd > best) { best = dd; bi = i; }
    }
    return bi;
}
static int support_index(int v0, int nv, int scb, int sck, ugk::gv d) {
    const int cell = scb >= 0 ? ugk_sc_cell(d.x, d.y, d.z, sck) : -1;
    if (cell < 0) return scan_first_max(v0, nullptr, nv, d);
    const unsigned short* L = &UG_SC_IDX[(scb + cell) * UG_SC_SLOTS];
    int cand[UG_FULL_HULL_MAXV], n = 0;
    if (L[0] == UG_SC_OVF) {
        const int cnt = L[1], off = L[2] | (L[3] << 16);
        for (int k = 0; k < cnt; k++) cand[n++] = UG_SC_IDX[off + k];
    } else {
        for (int k = 0; k < UG_SC_SLOTS; k++) cand[n++] = L[k];
    }
    return scan_first_max(v0, cand, n, d);
}
UGK_FN ugk::gv ugk_hull_support(const ugk::GShape& s, ugk::gv d) {
    const double* p = &UG_HULL_V[3 * (s.v0 + support_index(s.v0, s.nv, s.scb, s.sck, d))];
    return ugk::V3(p[0], p[1], p[2]);
}
/* a hull's support-cell table by its vertex range (the full hulls'), or -1 */
static void table_of(int v0, int nv, int& scb, int& sck) {
    scb = -1;
    sck = 0;
    for (int k = 0; k < UG_NSHAPE; k++)
        if (UG_SHAPE_KIND[k] == 1 && UG_SHAPE_FV0[k] == v0 && UG_SHAPE_FNV[k] == nv && nv > 0) {
            scb = UG_SHAPE_SCB[k];
            sck = UG_SHAPE_SCK[k];
        }
}
/* tests/test_supcells.py: the support index of n directions (xyz rows) for full-hull shape si, through the table
 * (use_table) or the whole scan */
extern "C" void ugk_host_support(int si, int use_table, int n, const double* dirs, int* out) {
    const int v0 = UG_SHAPE_FV0[si], nv = UG_SHAPE_FNV[si];
    const int scb = use_table ? UG_SHAPE_SCB[si] : -1, sck = UG_SHAPE_SCK[si];
    for (int k = 0; k < n; k++) out[k] = support_index(v0, nv, scb, sck, ugk::V3(dirs[3 * k], dirs[3 * k + 1], dirs[3 * k + 2]));
}
/* the cell a direction falls in (tests/test_supcells.py checks the classification against the numpy statement) */
extern "C" int ugk_host_cell(double x, double y, double z, int K) { return ugk_sc_cell(x, y, z, K); }

UGK_FN ugk::EFace ugk_face_get(ugk::EpaMem* E, int f) { return E->fc[f]; }
UGK_FN void ugk_face_put(ugk::EpaMem* E, int f, const ugk::EFace& F) { E->fc[f] = F; }
UGK_FN void ugk_face_pass(ugk::EpaMem* E, int f, int pass) { E->fc[f].pass = (unsigned char)pass; }
UGK_FN void ugk_face_link(ugk::EpaMem* E, int f, int j, int nf, int ne) {
    E->fc[f].f[j] = (unsigned char)nf;
    ugk::set_fe(E->fc[f], j, ne);
}
UGK_FN ugk::EHull ugk_hull_get(ugk::EpaMem* E, int i) { return E->hl[i]; }
UGK_FN void ugk_hull_put(ugk::EpaMem* E, int i, const ugk::EHull& h) { E->hl[i] = h; }
UGK_FN unsigned char* ugk_hpos(ugk::EpaMem* E) { return E->hpos; }
UGK_FN ugk::ESv ugk_svl_get(ugk::EpaMem* E, int i) { return E->sv[i]; }
UGK_FN void ugk_svl_put(ugk::EpaMem* E, int i, const ugk::ESv& v) { E->sv[i] = v; }
UGK_FN void ugk_ls_put(int* mem, ugk::LStack&, int i, int v) { mem[i] = v; }
UGK_FN int ugk_ls_get(const int* mem, const ugk::LStack&, int i) { return mem[i]; }
/* m_hull's first minimum of d * d over the hull array: the largest stamp among the minima; a NaN at the root (the
 * largest stamp) wins */
UGK_FN int ugk_epa_findbest(const ugk::EpaMem* E, int hcount) {
    const ugk::EHull* h = E->hl; /* the host keeps every hull slot in E */
    int root = 0;
    for (int i = 1; i < hcount; i++)
        if (h[i].stamp > h[root].stamp) root = i;
    double mind = h[root].d * h[root].d;
    if (mind != mind) return h[root].f;
    int best = root;
    for (int i = 0; i < hcount; i++) {
        const double sqd = h[i].d * h[i].d;
        if (sqd < mind || (sqd == mind && h[i].stamp > h[best].stamp)) { best = i; mind = sqd; }
    }
    return h[best].f;
}

static ugk::EpaMem g_epa;

/* shape: kind, v0, nv, imp[3], margin; pose: R (row-major 9), p (3).  out: n[3], pB[3], d.  Returns 1 with a point. */
extern "C" int ugk_host_pair(int kA, int v0A, int nvA, const double* impA, double mA, const double* RA, const double* pA,
                             int kB, int v0B, int nvB, const double* impB, double mB, const double* RB, const double* pB,
                             double thr, double* out) {
    ugk::GShape A{kA, v0A, nvA, ugk::V3(impA[0], impA[1], impA[2]), mA, -1, 0};
    ugk::GShape B{kB, v0B, nvB, ugk::V3(impB[0], impB[1], impB[2]), mB, -1, 0};
    if (kA == UG_SHAPE_HULL) table_of(v0A, nvA, A.scb, A.sck);
    if (kB == UG_SHAPE_HULL) table_of(v0B, nvB, B.scb, B.sck);
    ugk::gx TA, TB;
    for (int i = 0; i < 9; i++) { TA.R.m[i] = RA[i]; TB.R.m[i] = RB[i]; }
    TA.p = ugk::V3(pA[0], pA[1], pA[2]);
    TB.p = ugk::V3(pB[0], pB[1], pB[2]);
    ugk::gv n, p;
    double d;
    if (!ugk::gjk_pair(&g_epa, A, TA, B, TB, thr, n, p, d)) return 0;
    out[0] = n.x; out[1] = n.y; out[2] = n.z;
    out[3] = p.x; out[4] = p.y; out[5] = p.z;
    out[6] = d;
    return 1;
}
