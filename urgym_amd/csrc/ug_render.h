/* ug_render.h -- the camera (Camera.shot() -> p.getCameraImage, utilities.py:62-89): ray casting of one env's
 * collision geometry through a pybullet view / projection matrix pair.  Shared verbatim by the CPU restatement
 * (oracle/ug_oracle.c, ugo_camera) and the HIP kernel (ug_capi.hip, k_camera), so both evaluate the same
 * operations in the same order (bit-identical FP64, -ffp-contract=off on both sides).
 *
 * Pixel (col i, row j) of a W x H image casts the ray through NDC (x, y) = ((2i - W) / W, -(2j - H) / H) -- the
 * inverse of the reference's own rgbd_2_world / rgbd_2_world_batch (utilities.py:76-107), so a depth read back
 * through those functions lands on the surface the ray hit.  The ray runs from the near plane (NDC z = -1,
 * t = 0) to the far plane (z = +1, t = 1) of inv(P V); the first surface with t in [0, 1] is kept:
 *   depth = 0.5 * (P V p).z / (P V p).w + 0.5 (OpenGL's depth-buffer value, float), 1 where nothing is hit;
 *   seg   = body code (+ ((link + 1) << 24) with UGR_SEG_LINK), -1 where nothing is hit;
 *   rgba  = the shape's flat colour times 0.3 + 0.7 |n . d| (a headlight), background white.
 * Deviations from PyBullet (documented in include/urgym.h): the collision shapes are drawn (PyBullet draws the
 * visual meshes; for the primitives they coincide, the robot's visual meshes are concave where its hulls are
 * not), without collision margin; TinyRenderer's lighting, shadows and textures are not modelled; a ray that
 * starts inside a shape does not see it.
 */
#ifndef UG_RENDER_H
#define UG_RENDER_H

#include "ug_detmath.h"

#define UGR_SEG_LINK 1 /* seg = body + ((link + 1) << 24), ER_SEGMENTATION_MASK_OBJECT_AND_LINKINDEX */
#define UGR_MISS 1.0e300

typedef struct {
    double PV[16];  /* P V, row-major (PV[4 r + c]) */
    double iPV[16]; /* its inverse, row-major */
} UgrCam;

/* pybullet returns both matrices as 16 floats in column-major order (element (r, c) at [4 c + r]).
 * Returns 0, or -1 when P V is singular. */
UG_HD int ugr_setup(const float* view16, const float* proj16, UgrCam* cam) {
    double A[16], B[16];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += (double)proj16[4 * k + r] * (double)view16[4 * c + k];
            A[4 * r + c] = s;
            cam->PV[4 * r + c] = s;
            B[4 * r + c] = r == c ? 1.0 : 0.0;
        }
    /* Gauss-Jordan with partial pivoting */
    for (int c = 0; c < 4; c++) {
        int piv = c;
        for (int r = c + 1; r < 4; r++)
            if (ug_fabs(A[4 * r + c]) > ug_fabs(A[4 * piv + c])) piv = r;
        if (A[4 * piv + c] == 0.0) return -1;
        if (piv != c)
            for (int k = 0; k < 4; k++) {
                double t = A[4 * c + k]; A[4 * c + k] = A[4 * piv + k]; A[4 * piv + k] = t;
                t = B[4 * c + k]; B[4 * c + k] = B[4 * piv + k]; B[4 * piv + k] = t;
            }
        const double d = A[4 * c + c];
        for (int k = 0; k < 4; k++) { A[4 * c + k] = A[4 * c + k] / d; B[4 * c + k] = B[4 * c + k] / d; }
        for (int r = 0; r < 4; r++) {
            if (r == c) continue;
            const double f = A[4 * r + c];
            for (int k = 0; k < 4; k++) {
                A[4 * r + k] = A[4 * r + k] - f * A[4 * c + k];
                B[4 * r + k] = B[4 * r + k] - f * B[4 * c + k];
            }
        }
    }
    for (int i = 0; i < 16; i++) cam->iPV[i] = B[i];
    return 0;
}

/* the ray of pixel (i, j): origin on the near plane, direction to the far plane (t in [0, 1]) */
UG_HD void ugr_ray(const UgrCam* cam, int i, int j, int W, int H, double o[3], double d[3]) {
    const double x = (double)(2 * i - W) / (double)W, y = -((double)(2 * j - H) / (double)H);
    double pn[4], pf[4];
    for (int r = 0; r < 4; r++) {
        const double* m = &cam->iPV[4 * r];
        const double b = m[0] * x + m[1] * y;
        pn[r] = (b - m[2]) + m[3];
        pf[r] = (b + m[2]) + m[3];
    }
    for (int k = 0; k < 3; k++) {
        o[k] = pn[k] / pn[3];
        d[k] = pf[k] / pf[3] - o[k];
    }
}

/* OpenGL depth-buffer value of world point p */
UG_HD double ugr_depth(const UgrCam* cam, const double p[3]) {
    const double* m = cam->PV;
    const double z = ((m[8] * p[0] + m[9] * p[1]) + m[10] * p[2]) + m[11];
    const double w = ((m[12] * p[0] + m[13] * p[1]) + m[14] * p[2]) + m[15];
    return 0.5 * (z / w) + 0.5;
}

/* ---- ray / shape entry (shape frame; o, d the ray, t >= 0 of the entry or UGR_MISS, n its outward normal) ---- */
UG_HD double ugr_box(const double o[3], const double d[3], const double h[3], double n[3]) {
    double t0 = -UGR_MISS, t1 = UGR_MISS;
    int ax = -1;
    for (int k = 0; k < 3; k++) {
        if (d[k] == 0.0) {
            if (o[k] < -h[k] || o[k] > h[k]) return UGR_MISS;
            continue;
        }
        double a = (-h[k] - o[k]) / d[k], b = (h[k] - o[k]) / d[k];
        if (a > b) { const double t = a; a = b; b = t; }
        if (a > t0) { t0 = a; ax = k; }
        if (b < t1) t1 = b;
    }
    if (ax < 0 || t0 > t1 || t0 < 0.0) return UGR_MISS;
    n[0] = n[1] = n[2] = 0.0;
    n[ax] = d[ax] > 0.0 ? -1.0 : 1.0;
    return t0;
}
UG_HD double ugr_sphere(const double o[3], const double d[3], double r, double n[3]) {
    const double a = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    const double b = (o[0] * d[0] + o[1] * d[1]) + o[2] * d[2];
    const double c = ((o[0] * o[0] + o[1] * o[1]) + o[2] * o[2]) - r * r;
    const double disc = b * b - a * c;
    if (disc < 0.0) return UGR_MISS;
    const double t = (-b - ug_sqrt(disc)) / a;
    if (t < 0.0) return UGR_MISS;
    for (int k = 0; k < 3; k++) n[k] = (o[k] + t * d[k]) / r;
    return t;
}
/* convex hull: faces (nx, ny, nz, off) with n . x <= off inside (Cyrus-Beck) */
UG_HD double ugr_hull(const double o[3], const double d[3], const double* F, int nf, double n[3]) {
    double t0 = -UGR_MISS, t1 = UGR_MISS;
    int fe = -1;
    for (int f = 0; f < nf; f++) {
        const double* p = F + 4 * f;
        const double num = p[3] - ((p[0] * o[0] + p[1] * o[1]) + p[2] * o[2]);
        const double den = (p[0] * d[0] + p[1] * d[1]) + p[2] * d[2];
        if (den == 0.0) {
            if (num < 0.0) return UGR_MISS;
        } else if (den < 0.0) {
            const double t = num / den;
            if (t > t0) { t0 = t; fe = f; }
        } else {
            const double t = num / den;
            if (t < t1) t1 = t;
        }
        if (t0 > t1) return UGR_MISS;
    }
    if (fe < 0 || t0 < 0.0) return UGR_MISS;
    n[0] = F[4 * fe]; n[1] = F[4 * fe + 1]; n[2] = F[4 * fe + 2];
    return t0;
}
/* cylinder about z: radius r, half height hh */
UG_HD double ugr_cyl(const double o[3], const double d[3], double r, double hh, double n[3]) {
    double t0 = -UGR_MISS, t1 = UGR_MISS;
    int side = 0;
    const double a = d[0] * d[0] + d[1] * d[1];
    const double c = (o[0] * o[0] + o[1] * o[1]) - r * r;
    if (a == 0.0) {
        if (c > 0.0) return UGR_MISS;
    } else {
        const double b = o[0] * d[0] + o[1] * d[1];
        const double disc = b * b - a * c;
        if (disc < 0.0) return UGR_MISS;
        const double s = ug_sqrt(disc);
        t0 = (-b - s) / a;
        t1 = (-b + s) / a;
        side = 1;
    }
    if (d[2] == 0.0) {
        if (o[2] < -hh || o[2] > hh) return UGR_MISS;
    } else {
        double za = (-hh - o[2]) / d[2], zb = (hh - o[2]) / d[2];
        if (za > zb) { const double t = za; za = zb; zb = t; }
        if (za > t0) { t0 = za; side = 0; }
        if (zb < t1) t1 = zb;
    }
    if (t0 > t1 || t0 < 0.0 || t0 == -UGR_MISS) return UGR_MISS;
    if (side) {
        n[0] = (o[0] + t0 * d[0]) / r; n[1] = (o[1] + t0 * d[1]) / r; n[2] = 0.0;
    } else {
        n[0] = 0.0; n[1] = 0.0; n[2] = d[2] > 0.0 ? -1.0 : 1.0;
    }
    return t0;
}

/* the shape's flat colour (rgb in [0, 1]) by body code (include/urgym.h: 0 robot, 1 + i task object i, 10 table,
 * 11 plane, 12 golf pitch, 13 the Box's walls) -- the reference's rgbaColor where it sets one (BallBalance paddle
 * [1, 0.5, 0] and ball [1, 1, 1], env_ball_balance_v0.py:180,196), plain tones elsewhere (unpinned) */
UG_HD void ugr_color(int task, int ent, int link, double rgb[3]) {
    double r = 0.6, g = 0.6, b = 0.6;
    if (ent == 0) { if (link >= 8) { r = 0.25; g = 0.25; b = 0.25; } else { r = 0.75; g = 0.75; b = 0.78; } }
    else if (ent == 10) { r = 0.55; g = 0.4; b = 0.25; }
    else if (ent == 11) { r = 0.9; g = 0.9; b = 0.9; }
    else if (ent == 12) { r = 0.2; g = 0.6; b = 0.2; }
    else if (ent == 13) { r = 0.5; g = 0.35; b = 0.2; }
    else if (task == 0) { if (ent == 1) { r = 1.0; g = 0.5; b = 0.0; } else { r = 1.0; g = 1.0; b = 1.0; } }
    else if (ent == 1) { r = 0.8; g = 0.2; b = 0.2; }
    else if (ent == 2) { r = 0.2; g = 0.3; b = 0.8; }
    else { r = 0.9; g = 0.8; b = 0.2; }
    rgb[0] = r; rgb[1] = g; rgb[2] = b;
}
UG_HD unsigned char ugr_u8(double v) {
    const double c = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
    return (unsigned char)(int)(c * 255.0 + 0.5);
}

/* a ray's slab interval against an axis-aligned box lo..hi (shape frame): 0 when it misses it or the box lies
 * entirely outside t in [0, tmax] */
UG_HD int ugr_slab(const double o[3], const double d[3], const double* lo, const double* hi, double tmax) {
    double t0 = 0.0, t1 = tmax;
    for (int k = 0; k < 3; k++) {
        if (d[k] == 0.0) {
            if (o[k] < lo[k] || o[k] > hi[k]) return 0;
            continue;
        }
        double a = (lo[k] - o[k]) / d[k], b = (hi[k] - o[k]) / d[k];
        if (a > b) { const double t = a; a = b; b = t; }
        if (a > t0) t0 = a;
        if (b < t1) t1 = b;
        if (t0 > t1) return 0;
    }
    return 1;
}
/* one shape in world pose (R row-major, p): transforms the ray into the shape frame; culls by the bounding sphere
 * (radius rad about the shape origin) -- also when the sphere's entry lies beyond `best`, the nearest hit so far,
 * which no point of the shape can then beat -- and, for a hull, by its vertices' box (box6: lo xyz, hi xyz);
 * then the entry test.  Returns t or UGR_MISS, the normal in world axes. */
UG_HD double ugr_shape(const double R[9], const double p[3], double rad, int kind, const double half[3],
                       const double* F, int nf, const double* box6, double best, const double o[3], const double d[3],
                       double nw[3]) {
    const double q[3] = {o[0] - p[0], o[1] - p[1], o[2] - p[2]};
    const double dd = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    const double tc = -((q[0] * d[0] + q[1] * d[1]) + q[2] * d[2]) / dd;
    const double e[3] = {q[0] + tc * d[0], q[1] + tc * d[1], q[2] + tc * d[2]};
    const double e2 = (e[0] * e[0] + e[1] * e[1]) + e[2] * e[2];
    if (e2 > rad * rad) return UGR_MISS;
    if (tc - ug_sqrt((rad * rad - e2) / dd) > best) return UGR_MISS;
    double os[3], ds[3], n[3];
    for (int k = 0; k < 3; k++) {
        os[k] = (R[k] * q[0] + R[3 + k] * q[1]) + R[6 + k] * q[2];
        ds[k] = (R[k] * d[0] + R[3 + k] * d[1]) + R[6 + k] * d[2];
    }
    double t;
    if (kind == 0) t = ugr_box(os, ds, half, n);
    else if (kind == 1) t = ugr_slab(os, ds, box6, box6 + 3, best < 1.0 ? best : 1.0) ? ugr_hull(os, ds, F, nf, n) : UGR_MISS;
    else if (kind == 2) t = ugr_sphere(os, ds, half[0], n);
    else t = ugr_cyl(os, ds, half[0], half[2], n);
    if (t == UGR_MISS || t > 1.0) return UGR_MISS;
    for (int k = 0; k < 3; k++) nw[k] = (R[3 * k] * n[0] + R[3 * k + 1] * n[1]) + R[3 * k + 2] * n[2];
    return t;
}
/* a hull's vertex box in its shape frame (box6: lo xyz, hi xyz) */
UG_HD void ugr_hull_box(const double* V, int nv, double box6[6]) {
    for (int k = 0; k < 3; k++) { box6[k] = UGR_MISS; box6[3 + k] = -UGR_MISS; }
    for (int v = 0; v < nv; v++)
        for (int k = 0; k < 3; k++) {
            const double x = V[3 * v + k];
            if (x < box6[k]) box6[k] = x;
            if (x > box6[3 + k]) box6[3 + k] = x;
        }
}
/* bounding radius of a shape about its origin (hull: its farthest vertex) */
UG_HD double ugr_radius(int kind, const double half[3], const double* V, int nv) {
    if (kind == 0) return ug_sqrt((half[0] * half[0] + half[1] * half[1]) + half[2] * half[2]);
    if (kind == 2) return half[0];
    if (kind == 3) return ug_sqrt(half[0] * half[0] + half[2] * half[2]);
    double m = 0.0;
    for (int v = 0; v < nv; v++) {
        const double* x = V + 3 * v;
        const double s = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
        if (s > m) m = s;
    }
    return ug_sqrt(m);
}
/* the pixel's outputs from its nearest hit (t, normal, shape) */
UG_HD void ugr_shade(const UgrCam* cam, int task, double t, const double nw[3], int ent, int link, int flags,
                     const double o[3], const double d[3], unsigned char* rgba, float* depth, int* seg) {
    if (t == UGR_MISS) {
        rgba[0] = rgba[1] = rgba[2] = rgba[3] = 255;
        *depth = 1.0f;
        *seg = -1;
        return;
    }
    const double p[3] = {o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]};
    *depth = (float)ugr_depth(cam, p);
    *seg = (flags & UGR_SEG_LINK) ? ent + ((link + 1) << 24) : ent;
    const double dl = ug_sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
    const double cs = ug_fabs((nw[0] * d[0] + nw[1] * d[1]) + nw[2] * d[2]) / dl;
    double c[3];
    ugr_color(task, ent, link, c);
    const double s = 0.3 + 0.7 * cs;
    rgba[0] = ugr_u8(c[0] * s); rgba[1] = ugr_u8(c[1] * s); rgba[2] = ugr_u8(c[2] * s); rgba[3] = 255;
}

#endif
