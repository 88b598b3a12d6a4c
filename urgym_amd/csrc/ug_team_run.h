/* ug_team_run.h -- part of ug_team.h: one substep (team_substep), the task glue, the env program (team_run), launch priority, state in / out.
 * Included by ug_team.h inside namespace ugd, in this order (the kernel is one translation unit); not self-contained. */
/* ---------------- one p.stepSimulation() (oracle substep()) ---------------- */
__device__ __forceinline__ static void team_substep(const Scene* s, double* ws) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    EnvState& e = sh.e;
#ifdef UG_PROF
    unsigned long long fsnap = lane < UG_FREE_SPLIT_N ? sh.prof[kFreeSplit[lane]] : 0ull; /* lane i: counter i */
#endif
    PROF_T0(t_col);
    PROF_PRE_CALL();
    serial_fk();
    PROF_POST_CALL(CS_FK);
    __syncthreads();
    PROF_ADD(PF_FK, t_col);
    const double ov0 = e.overflow;
    if (s->gjk) {
        if (s->full) {
            if (!(uniform(sh.qsvalid) && quiescent_ok(s, ws))) {
                PROF_PRE_CALL();
                team_collide<true, true>(s, ws);
                PROF_POST_CALL(CS_COLLIDE);
            } else PROF_CNT(PC_QUIET, 1);
        } else team_collide<false, true>(s, ws);
    } else {
        if (s->full) team_collide<true, false>(s, ws);
        else team_collide<false, false>(s, ws);
    }
    const double ov1 = e.overflow;
    if (lane == 0) {
        sh.stats[UG_STAT_SUBSTEPS]++;
        if (ov1 != ov0) { sh.stats[UG_STAT_MANCAP]++; sh.flags |= UG_FLAG_DROPPED; }
    }
    PROF_ADD(PF_COLLIDE, t_col);
    PROF_T0(t_dyn);
    PROF_PRE_CALL();
    serial_pre(s);
    PROF_POST_CALL(CS_PRE);
    __syncthreads();
    if (lane == 0 && e.overflow != ov1) { sh.stats[UG_STAT_ROWCAP]++; sh.flags |= UG_FLAG_DROPPED; }
    PROF_ADD(PF_DYN, t_dyn);
    PROF_T0(t_rows);
    const int n = uniform(sh.nrows), nnc = uniform(sh.nnc), nn = uniform(sh.nn);
    PROF_CNT(PC_SUBSTEPS, 1);
    PROF_CNT(PC_ROWS, n);
    PROF_CNT(PC_NNC, nnc);
    PROF_CNT(PC_NN, nn);
    PROF_CNT(PC_N64, n <= 64);
    PROF_CNT(PC_N80, n > 64 && n <= 80);
    PROF_CNT(PC_N96, n > 80 && n <= 96);
    PROF_CNT(PC_OVL, sh.nov);
    PROF_CNT(PC_NMAN, (int)e.nman);
    /* rows: built lane-per-row into the workspace (J | M^-1 J^T) and LDS (scalars) */
    PROF_T0(t_unit);
    PROF_PRE_CALL();
    team_unit_solves();
    PROF_POST_CALL(CS_UNIT);
    PROF_ADD(PF_UNIT, t_unit);
    PROF_T0(t_rowb);
    /* the motor / gear solve (team_pgs's direct path) reads its Delassus rows and M^-1 J^T from the unit
     * solves in LDS: its J | M^-1 J^T stay out of the workspace */
#ifdef UG_DEBUG_DUMP
    const bool nc_direct = false;
#else
    const bool nc_direct = n == 12 && nnc == 12 && ballot(lane < 12 && sh.rs[lane].kind == 0) == 0ull;
#endif
#ifdef UG_INLINE_ROWS /* A/B aid: the row build inlined into the kernel as before round 6 */
    for (int p = lane; p < n; p += TEAM) build_row(s, p, ws + WS_ROWS + p * RS, !nc_direct);
#else
    team_build_rows(s, n, ws, !nc_direct);
#endif
    PROF_ADD(PF_ROWB, t_rowb);
    __threadfence_block();
    __syncthreads();
    PROF_ADD(PF_ROWS, t_rows);
    PROF_T0(t_pgs);
    double dv, dvs;
    PROF_PRE_CALL();
    int split = team_pgs(ws, n, nnc, nn, s->nobj, dv, dvs);
    PROF_POST_CALL(CS_PGS);
    if (lane == 0 && split) sh.stats[UG_STAT_SPLIT]++;
    PROF_ADD(PF_PGS, t_pgs);
    PROF_T0(t_int);
    if (lane < NVP) { sh.dvout[lane] = dv; sh.dvsout[lane] = dvs; }
    /* impulses back into the manifold points (lane per row) */
    for (int p = nnc + lane; p < n; p += TEAM) {
        const RowS& r = sh.rs[p];
        StPt& pt = e.man[r.a].pt[r.b];
        if (r.kind == 3) pt.imp = r.imp;
        else if (r.kind == 4) pt.imp1 = r.imp;
        else if (r.kind == 5) pt.imp2 = r.imp;
    }
    __syncthreads();
    PROF_PRE_CALL();
    serial_post(s, split);
    PROF_POST_CALL(CS_POST);
    __syncthreads();
    PROF_ADD(PF_INTEG, t_int);
#ifdef UG_PROF
    if (n == 12 && nnc == 12) { /* contact-free substeps (most of a reset's settling) on their own */
        PROF_CNT(PC_FREE, 1);
        PROF_CNT(PF_FREE_COL, t_dyn - t_col);
        PROF_CNT(PF_FREE_DYN, t_rows - t_dyn);
        PROF_CNT(PF_FREE_ROWS, t_pgs - t_rows);
        PROF_CNT(PF_FREE_PGS, t_int - t_pgs);
        PROF_ADD(PF_FREE_INT, t_int);
    }
    __syncthreads();
    if (n == 12 && nnc == 12 && lane < UG_FREE_SPLIT_N) sh.prof[PF_FREE_SUB0 + lane] += sh.prof[kFreeSplit[lane]] - fsnap;
    __syncthreads();
#endif
}

/* ---------------- robot control + BallBalance glue (lane 0 unless noted) ---------------- */
__device__ static inline void set_gripper(EnvState& e, double L) {
    e.mtarget[6] = gripper_angle(L);
    e.mon[6] = 1.0;
}
__device__ static inline void open_gripper(EnvState& e, double pct) {
    set_gripper(e, UG_GRIP_MIN + (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0));
}
__device__ static inline void close_gripper(EnvState& e, double pct) {
    set_gripper(e, UG_GRIP_MAX - (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0));
}
__device__ static void move_ee_end(EnvState& e, v3 pos, q4 orn) {
    double qt[NB];
    ik_solve(e.q, pos, orn, qt);
    for (int i = 0; i < 6; i++) { e.mtarget[i] = qt[i]; e.mon[i] = 1.0; }
}
__device__ static void link_state_of(const double* q, int l, v3& p, q4& o) {
    Kin k;
    fk(q, k);
    m3 R;
    link_frame(k, l, 1, R, p);
    o = mquat(R);
}
__device__ static v3 gripper_center(const double* q) {
    Kin k;
    fk(q, k);
    v3 lo = V(1e300, 1e300, 1e300), hi = V(-1e300, -1e300, -1e300);
    const int links[2] = {11, 16};
    for (int i = 0; i < 2; i++) {
        int l = links[i];
        m3 R;
        v3 p;
        link_frame(k, l, 1, R, p);
        v3 c = vadd(mv(R, V(UG_LINK_AABB_C[3 * l], UG_LINK_AABB_C[3 * l + 1], UG_LINK_AABB_C[3 * l + 2])), p);
        v3 hh = V(UG_LINK_AABB_H[3 * l], UG_LINK_AABB_H[3 * l + 1], UG_LINK_AABB_H[3 * l + 2]);
        const double* r = R.m;
        v3 ext = V(ug_fabs(r[0]) * hh.x + ug_fabs(r[1]) * hh.y + ug_fabs(r[2]) * hh.z,
                   ug_fabs(r[3]) * hh.x + ug_fabs(r[4]) * hh.y + ug_fabs(r[5]) * hh.z,
                   ug_fabs(r[6]) * hh.x + ug_fabs(r[7]) * hh.y + ug_fabs(r[8]) * hh.z);
        v3 mn = vsub(c, ext), mx = vadd(c, ext);
        lo = V(ug_min(lo.x, mn.x), ug_min(lo.y, mn.y), ug_min(lo.z, mn.z));
        hi = V(ug_max(hi.x, mx.x), ug_max(hi.y, mx.y), ug_max(hi.z, mx.z));
    }
    return V((hi.x + lo.x) / 2.0, (hi.y + lo.y) / 2.0, (hi.z + lo.z) / 2.0);
}
__device__ static void drop_manifolds_of(EnvState& e, const Scene* s, int c0, int c1) {
    int k = 0, nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if ((P.a >= c0 && P.a < c1) || (P.b >= c0 && P.b < c1)) continue;
        if (k != m) e.man[k] = e.man[m];
        k++;
    }
    e.nman = (double)k;
}
__device__ static void remove_object(EnvState& e, const Scene* s, int o) {
    e.oactive[o] = 0.0;
    int c0 = s->ocol[o], c1 = c0 + s->oncol[o];
    int k = 0, nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if ((P.a >= c0 && P.a < c1) || (P.b >= c0 && P.b < c1)) continue;
        if (k != m) e.man[k] = e.man[m];
        k++;
    }
    e.nman = (double)k;
}
__device__ static void place_object(EnvState& e, int o, v3 pos, q4 orn) {
    e.oactive[o] = 1.0;
    e.obj[o].pos = pos;
    e.obj[o].quat = orn;
    e.obj[o].v = V(0, 0, 0);
    e.obj[o].w = V(0, 0, 0);
}
/* random.uniform(a, b) from the env's stream, or from a caller-supplied draw in [0,1) */
struct Draws {
    Rng rng;
    const double* given;
    int k;
    /* one random.random(): the caller's reset draw when given, else the env's MT19937 stream */
    __device__ double next() { return given ? given[k++] : mt_random(rng); }
    __device__ double uniform(double a, double b) { return ugg_uniform(a, b, next()); }
};
__device__ static void bb_obs(const EnvState& e, double* obs) {
    v3 eu = euler_from_quat(e.obj[0].quat);
    obs[0] = eu.x; obs[1] = eu.y; obs[2] = eu.z;
    obs[3] = e.obj[0].pos.x - e.obj[1].pos.x;
    obs[4] = e.obj[0].pos.y - e.obj[1].pos.y;
    obs[5] = e.obj[0].pos.z - e.obj[1].pos.z;
}
/* p.getContactPoints existence: a manifold point between a robot link in [lmin, lmax]
 * and collider cb (robot colliders are always side A of their pairs) */
__device__ static int robot_contact(const EnvState& e, const Scene* s, int cb, int lmin, int lmax) {
    int nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if (e.man[m].npts <= 0.0 || P.b != cb) continue;
        int l = s->col[P.a].link;
        if (l >= lmin && l <= lmax) return 1;
    }
    return 0;
}
__device__ static int static_collider(const Scene* s, int ent) {
    for (int i = 0; i < s->ncol; i++)
        if (s->col[i].ent == ent) return i;
    return -1;
}
__device__ static void move_ee_joint(EnvState& e, const double* q6) {
    for (int i = 0; i < 6; i++) { e.mtarget[i] = q6[i]; e.mon[i] = 1.0; }
}
/* CubesPush obs (env_cubes_push_v0.py:196-205) */
__device__ static void cp_obs(const EnvState& e, double* obs) {
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    obs[0] = pe.x; obs[1] = pe.y; obs[2] = pe.z;
    for (int o = 0; o < 2; o++) { obs[3 + 3 * o] = e.obj[o].pos.x; obs[4 + 3 * o] = e.obj[o].pos.y; obs[5 + 3 * o] = e.obj[o].pos.z; }
}
/* CubesGrasp: opening from link frames 11/16 (env_cubes_grasp_v0.py:349-376) */
__device__ static double cg_opening(const EnvState& e) {
    Kin k;
    fk(e.q, k);
    m3 R1, R2;
    v3 p1, p2;
    link_frame(k, 11, 0, R1, p1);
    link_frame(k, 16, 0, R2, p2);
    return ugg_cg_opening(ug_norm3(p2.x - p1.x, p2.y - p1.y, p2.z - p1.z));
}
__device__ static void cg_obs(const EnvState& e, double* obs) {
    /* :268-287 */
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    obs[0] = e.goal_approached; obs[1] = e.goal_grasped;
    obs[2] = pe.x; obs[3] = pe.y; obs[4] = pe.z; obs[5] = oe.x; obs[6] = oe.y; obs[7] = oe.z; obs[8] = oe.w;
    obs[9] = cg_opening(e);
    obs[10] = e.obj[0].pos.x; obs[11] = e.obj[0].pos.y; obs[12] = e.obj[0].pos.z;
    obs[13] = e.obj[0].quat.x; obs[14] = e.obj[0].quat.y; obs[15] = e.obj[0].quat.z; obs[16] = e.obj[0].quat.w;
}
/* Golf: any manifold point between colliders [a0, a1) and [b0, b1) (either side of the pair) */
__device__ static int pair_contact(const EnvState& e, const Scene* s, int a0, int a1, int b0, int b1) {
    int nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if (e.man[m].npts <= 0.0) continue;
        if ((P.a >= a0 && P.a < a1 && P.b >= b0 && P.b < b1) || (P.b >= a0 && P.b < a1 && P.a >= b0 && P.a < b1))
            return 1;
    }
    return 0;
}
/* club reference point at base-frame height zoff: composite COM + R (0, 0, zoff - zc) */
__device__ static v3 club_point(const EnvState& e, double zoff) {
    m3 R = qmat(e.obj[0].quat);
    return vadd(e.obj[0].pos, mv(R, V(0.0, 0.0, zoff - UG_GF_ZC)));
}
__device__ static void gf_obs(const EnvState& e, double* obs) {
    v3 st = club_point(e, UG_GF_FOOT_Z);
    double stick[3] = {st.x, st.y, st.z}, ball[3] = {e.obj[1].pos.x, e.obj[1].pos.y, e.obj[1].pos.z};
    double hole[3] = {UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z};
    ugg_gf_obs(stick, ball, hole, obs);
}
/* CubesPushDiff obs (env_cubes_push_diff_v0.py:202-212): ee position, each cube minus the ee position */
__device__ static void cpd_obs(const EnvState& e, double* obs) {
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    obs[0] = pe.x; obs[1] = pe.y; obs[2] = pe.z;
    for (int o = 0; o < 2; o++) {
        obs[3 + 3 * o] = e.obj[o].pos.x - pe.x; obs[4 + 3 * o] = e.obj[o].pos.y - pe.y; obs[5 + 3 * o] = e.obj[o].pos.z - pe.z;
    }
}
/* TwoBallsBalance obs (env_two_balls_balance_v0.py:157-163): paddle euler, paddle - ball 1, paddle - ball 2 */
__device__ static void tb_obs(const EnvState& e, double* obs) {
    v3 eu = euler_from_quat(e.obj[0].quat);
    obs[0] = eu.x; obs[1] = eu.y; obs[2] = eu.z;
    for (int b = 0; b < 2; b++) {
        obs[3 + 3 * b] = e.obj[0].pos.x - e.obj[1 + b].pos.x;
        obs[4 + 3 * b] = e.obj[0].pos.y - e.obj[1 + b].pos.y;
        obs[5 + 3 * b] = e.obj[0].pos.z - e.obj[1 + b].pos.z;
    }
}
/* non-finite state guard (oracle state_finite): q, qd and the active objects' state */
__device__ static int state_finite(const Scene* s, const EnvState& e) {
    for (int i = 0; i < NB; i++)
        if (!__builtin_isfinite(e.q[i]) || !__builtin_isfinite(e.qd[i])) return 0;
    for (int o = 0; o < s->nobj; o++) {
        if (e.oactive[o] == 0.0) continue;
        const double* v = &e.obj[o].pos.x;
        for (int j = 0; j < UG_OBJ_DOUBLES; j++)
            if (!__builtin_isfinite(v[j])) return 0;
    }
    return 1;
}
/* a reset of a non-finite state starts from a clean robot (oracle sanitize) */
__device__ static void sanitize(const Scene* s, EnvState& e) {
    if (state_finite(s, e)) return;
    for (int i = 0; i < NB; i++) { e.q[i] = 0.0; e.qd[i] = 0.0; }
    for (int m = 0; m < 7; m++) { e.mtarget[m] = 0.0; e.mon[m] = 0.0; }
    for (int o = 0; o < MAXOBJ; o++) {
        e.oactive[o] = 0.0;
        e.obj[o].pos = V(0, 0, 0); e.obj[o].quat = Q(0, 0, 0, 0); e.obj[o].v = V(0, 0, 0); e.obj[o].w = V(0, 0, 0);
    }
    e.nman = 0.0;
}
/* ---- Box (env_box_v0.py; oracle bx_*) ---- */
/* get_ee_pose() in world coordinates: the robot base stands at (0, UG_BX_ROBOT_Y, 0) */
__device__ __forceinline__ static void bx_ee_world(const EnvState& e, double* w7) {
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    w7[0] = pe.x; w7[1] = pe.y + UG_BX_ROBOT_Y; w7[2] = pe.z;
    w7[3] = oe.x; w7[4] = oe.y; w7[5] = oe.z; w7[6] = oe.w;
}
/* move_ee(world pose, 'end'): the target taken into the base frame (position shifted back, orientation through
 * btMatrix3x3 setRotation / getRotation) */
__device__ static void bx_move_ee(EnvState& e, const double* w7) {
    const m3 R = qmat(Q(w7[3], w7[4], w7[5], w7[6]));
    move_ee_end(e, V(w7[0], w7[1] - UG_BX_ROBOT_Y, w7[2]), mquat(R));
}
/* reset_box (:172-177): both joints to 0 at rest, the link frames follow */
__device__ static void bx_place(const Scene* s, EnvState& e) {
    for (int o = 0; o < 2; o++) {
        e.oactive[o] = 1.0;
        e.obj[o].v = V(0, 0, 0);
        e.obj[o].w = V(0, 0, 0);
        double qt[4], pt[3];
        ugj_frame(&s->ojoint[o], 0.0, qt, pt);
        e.obj[o].quat = Q(qt[0], qt[1], qt[2], qt[3]);
        e.obj[o].pos = V(pt[0], pt[1], pt[2]);
    }
}
__device__ static void task_obs(const Scene* s, const EnvState& e, double* obs) {
    if (s->task == UG_TASK_BOX) bx_ee_world(e, obs); /* :161-170 np.array(ee_pos) */
    else if (s->variant == UG_TASK_TWOBALLS) tb_obs(e, obs);
    else if (s->variant == UG_TASK_CUBESPUSHDIFF) cpd_obs(e, obs);
    else if (s->task == UG_TASK_CUBESPUSH) cp_obs(e, obs);
    else if (s->task == UG_TASK_CUBESGRASP) cg_obs(e, obs);
    else if (s->variant == UG_TASK_GOLFJOINTS) { /* env_golf_joints_v0.py:228-235: arm joints, then the Golf obs */
        for (int i = 0; i < 6; i++) obs[i] = e.q[i];
        gf_obs(e, obs + 6);
    } else if (s->task == UG_TASK_GOLF) gf_obs(e, obs);
    else bb_obs(e, obs);
}
/* ---------------- the env program: step / reset as one substep loop ----------------
 * The reference's control flow (env_ball_balance_v0.py: step 105-134, reset 145-170, wait_until_stable
 * 94-103, robot.reset 89-106) is a sequence of glue actions separated by physics loops.  It runs here as
 * a small state machine around a single inlined team_substep(), so the PGS register slots exist once. */
enum { G_STEP = 0, G_STEP_DONE, G_RESET, G_RESET_ROBOT, G_RESET_PLACE, G_RESET_DONE, G_END };
enum { L_NONE = 0, L_FIXED10, L_WAIT, L_FIXED120 };
struct RunIO {
    const float* act;    /* step action (task act_dim floats) */
    double* obs;         /* obs row */
    double* final_obs;   /* final obs row (autoreset) or null */
    Draws dr;            /* reset draws */
    int autoreset, trunc;
    double rew;
    int term, succ, reset_done;
};
/* lane-0 glue of one program point; returns the physics loop to run next and sets *next */
__device__ __noinline__ static int glue(const Scene* s, int pc, RunIO& io, int* next) {
    PROF_CALL(CALL_GLUE);
    EnvState& e = g_sh.e;
    const int task = s->task;
    const int O = UG_OBS_DIM(s->variant);
    switch (pc) {
        case G_STEP: {
            v3 pe;
            q4 oe;
            if (task == UG_TASK_BOX) { /* env_box_v0.py:125-129: ee pose + action, the gripper, 120 substeps */
                double w7[7], t7[7];
                bx_ee_world(e, w7);
                ugg_box_target(w7, io.act, t7);
                bx_move_ee(e, t7);
                e.mtarget[6] = gripper_angle((double)io.act[7]); /* move_gripper(action[-1]) */
                e.mon[6] = 1.0;
                *next = G_STEP_DONE;
                return L_FIXED120;
            }
            if (task == UG_TASK_CUBESGRASP) {
                /* env_cubes_grasp_v0.py:132-158: random.choices picks joint move or gripper command */
                int sel = ugg_cg_choose(io.act[0], io.act[1], io.dr.next());
                if (sel == 0) {
                    double q6[6];
                    for (int i = 0; i < 6; i++) q6[i] = (double)io.act[2 + i];
                    move_ee_joint(e, q6);
                } else if (io.act[8] < 0.5f) {
                    open_gripper(e, 100.0);
                } else {
                    close_gripper(e, 100.0);
                }
            } else if (task == UG_TASK_CUBESPUSH) {
                /* env_cubes_push_v0.py:115-127: EE position + action, vertical orientation */
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                move_ee_end(e, V(pe.x + (double)io.act[0], pe.y + (double)io.act[1], pe.z + (double)io.act[2]),
                            Q(0.0, UG_VQ_S, 0.0, UG_VQ_C));
            } else if (s->variant == UG_TASK_GOLFJOINTS) {
                /* env_golf_joints_v0.py:122-124: arm joint positions + action (float64 + float32 -> float64),
                 * move_ee(..., 'joint') */
                double q6[6];
                for (int i = 0; i < 6; i++) q6[i] = e.q[i] + (double)io.act[i];
                move_ee_joint(e, q6);
            } else if (task == UG_TASK_GOLF) {
                /* env_golf_v0.py:115-127: EE position + action, the reset orientation (0, 0, -0.7, 0.7) */
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                move_ee_end(e, V(pe.x + (double)io.act[0], pe.y + (double)io.act[1], pe.z + (double)io.act[2]),
                            Q(0.0, 0.0, -0.70, 0.70));
            } else {
                /* env_ball_balance_v0.py:105-118: move_ee(end pose + action on the euler angles) */
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                v3 eu = euler_from_quat(oe);
                eu.x += (double)io.act[0]; eu.y += (double)io.act[1]; eu.z += (double)io.act[2];
                move_ee_end(e, pe, quat_from_euler(eu));
            }
            *next = G_STEP_DONE;
            return L_WAIT;
        }
        case G_STEP_DONE:
            if (task == UG_TASK_CUBESPUSH) { /* :129-150 */
                int table = robot_contact(e, s, static_collider(s, 10), 1, UG_NL - 1);
                int touched = robot_contact(e, s, s->ocol[1], 9, 18);
                io.succ = ugg_cp_reward(table, touched, e.obj[0].pos.x, e.obj[0].pos.y, e.obj[0].pos.z, e.obj[1].pos.x,
                                        e.obj[1].pos.y, e.obj[1].pos.z, s->sparse, &io.rew);
                io.term = io.succ;
            } else if (task == UG_TASK_CUBESGRASP) { /* :160-192 */
                v3 gc = gripper_center(e.q);
                double d = ug_norm3(gc.x - e.obj[0].pos.x, gc.y - e.obj[0].pos.y, gc.z - e.obj[0].pos.z);
                int grasp = robot_contact(e, s, s->ocol[0], 11, 13) && robot_contact(e, s, s->ocol[0], 16, 18);
                int app = (int)e.goal_approached, gr = (int)e.goal_grasped;
                io.succ = ugg_cg_reward(&app, &gr, d, cg_opening(e), grasp, e.obj[0].pos.z, &io.rew);
                e.goal_approached = (double)app;
                e.goal_grasped = (double)gr;
                io.term = io.succ;
            } else if (task == UG_TASK_GOLF) { /* env_golf_v0.py:129-183 */
                int c0 = s->ocol[0], c1 = c0 + s->oncol[0], cb = s->ocol[1], cp = static_collider(s, 12);
                int in_fingers = 0;
                for (int c = c0; c < c1; c++) in_fingers |= robot_contact(e, s, c, 9, 18);
                int floor = robot_contact(e, s, cp, 0, UG_NL - 1) || pair_contact(e, s, c0, c1, cp, cp + 1);
                int touched = pair_contact(e, s, cb, cb + 1, c0, c1);
                v3 st = club_point(e, UG_GF_FOOT_Z);
                double stick[3] = {st.x, st.y, st.z}, ball[3] = {e.obj[1].pos.x, e.obj[1].pos.y, e.obj[1].pos.z};
                double hole[3] = {UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z};
                io.succ = ugg_gf_reward(ball, hole, stick, in_fingers, floor, touched, s->sparse, &io.rew, &io.term);
            } else if (task == UG_TASK_BOX) { /* env_box_v0.py:131-139, update_reward :141-159 */
                const int bc = s->ocol[1];
                int press = ugg_box_press(e.obj[1].w.x, s->button_mode, robot_contact(e, s, bc, 0, UG_NL - 1),
                                          robot_contact(e, s, bc, 9, 18));
                int op = (int)e.goal_approached, pr = (int)e.goal_grasped, cl = (int)e.spare;
                io.term = ugg_box_reward(&op, &pr, &cl, e.obj[0].w.x, press, &io.rew);
                e.goal_approached = (double)op;
                e.goal_grasped = (double)pr;
                e.spare = (double)cl;
                io.succ = io.term;
            } else if (s->variant == UG_TASK_TWOBALLS) { /* env_two_balls_balance_v0.py:110-146 */
                double b1[3] = {e.obj[1].pos.x, e.obj[1].pos.y, e.obj[1].pos.z};
                double b2[3] = {e.obj[2].pos.x, e.obj[2].pos.y, e.obj[2].pos.z};
                io.term = ugg_tb_reward(io.act, b1, b2, e.obj[0].pos.z, &io.rew);
                io.succ = 0;
            } else { /* env_ball_balance_v0.py:119-134: reward 1, terminated when the ball falls below the paddle */
                io.rew = 1.0;
                io.term = e.obj[1].pos.z < e.obj[0].pos.z;
                io.succ = 0;
            }
            if (!state_finite(s, e)) { /* end the episode, zero reward; the autoreset restarts from a clean state */
                io.term = 1;
                io.succ = 0;
                io.rew = 0.0;
                g_sh.flags |= UG_FLAG_NONFINITE;
                g_sh.stats[UG_STAT_NONFINITE]++;
            }
            task_obs(s, e, io.obs);
            if (io.autoreset && (io.term || io.trunc)) {
                if (io.final_obs)
                    for (int j = 0; j < O; j++) io.final_obs[j] = io.obs[j];
                *next = G_RESET;
                return L_NONE;
            }
            *next = G_END;
            return L_NONE;
        case G_RESET: /* robot.reset(): reset_arm (rest pose) + 10 substeps */
            sanitize(s, e);
            e.goal_approached = 0.0;
            e.goal_grasped = 0.0;
            e.spare = 0.0; /* Box: box_closed */
            for (int i = 0; i < 6; i++) { e.q[i] = UG_ARM_REST[i]; e.qd[i] = 0.0; }
            *next = G_RESET_ROBOT;
            return L_FIXED10;
        case G_RESET_ROBOT: /* reset_gripper (open 100), then the task's scene and start pose */
            open_gripper(e, 100.0);
            if (task == UG_TASK_BOX) { /* env_box_v0.py:181-184: move_ee(get_ee_pose(), 'end'), reset_box(); no settling */
                double w7[7];
                bx_ee_world(e, w7);
                bx_move_ee(e, w7);
                bx_place(s, e);
                *next = G_RESET_DONE;
                return L_NONE;
            }
            for (int o = 0; o < s->nobj; o++) remove_object(e, s, o);
            if (task == UG_TASK_CUBESPUSH) { /* env_cubes_push_v0.py:207-227, create_cubes :240-246 */
                place_object(e, 0, V(0.0, -0.5, 0.1), Q(0, 0, 0, 1));
                double x = ugg_cp_cube1_x(io.dr.next());
                place_object(e, 1, V(x, -0.7, 0.1), Q(0, 0, 0, 1));
                move_ee_end(e, V(x, -0.7, 0.1 + UG_CP_EE_DZ), Q(0.0, UG_VQ_S, 0.0, UG_VQ_C));
                close_gripper(e, 100.0);
                *next = G_RESET_DONE;
            } else if (task == UG_TASK_CUBESGRASP) { /* env_cubes_grasp_v0.py:289-307, create_cubes :310-330 */
                double u0 = io.dr.next(), u1 = io.dr.next(), x, y;
                ugg_cg_cube_xy(u0, u1, &x, &y);
                place_object(e, 0, V(x, y, 0.1), Q(0, 0, 0, 1));
                v3 pe;
                q4 oe;
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                move_ee_end(e, pe, oe);
                *next = G_RESET_DONE;
            } else if (task == UG_TASK_GOLF) { /* env_golf_v0.py:238-252: pitch re-created, start pose, open 20% */
                int cp = static_collider(s, 12);
                drop_manifolds_of(e, s, cp, cp + 1);
                move_ee_end(e, V(0.0, -0.60, 0.40), Q(0.0, 0.0, -0.70, 0.70));
                open_gripper(e, 20.0);
                *next = G_RESET_PLACE;
            } else { /* env_ball_balance_v0.py:145-160: move_ee(start pose); open 20% */
                move_ee_end(e, V(0.0, -0.60, 0.60), Q(0.50, -0.50, -0.50, 0.50));
                open_gripper(e, 20.0);
                *next = G_RESET_PLACE;
            }
            return L_WAIT;
        case G_RESET_PLACE: { /* BallBalance: paddle between the fingers, ball above it; close gripper */
            if (task == UG_TASK_GOLF) { /* env_golf_v0.py:254-265: club under the gripper centre, ball; close */
                v3 gc = gripper_center(e.q);
                place_object(e, 0, V(gc.x, gc.y, gc.z - 0.05 + UG_GF_ZC), Q(0, 0, 0, 1));
                double u0 = io.dr.next(), u1 = io.dr.next(), bx, by;
                ugg_gf_ball_xy(u0, u1, &bx, &by);
                place_object(e, 1, V(bx, by, 0.1), Q(0, 0, 0, 1));
                close_gripper(e, 100.0);
                *next = G_RESET_DONE;
                return L_WAIT;
            }
            v3 pe;
            q4 oe;
            link_state_of(e.q, UG_EE_LINK, pe, oe);
            v3 gc = gripper_center(e.q);
            v3 pose = V(pe.x, pe.y - 0.2, gc.z);
            place_object(e, 0, pose, Q(0, 0, 0, 1));
            if (s->variant == UG_TASK_TWOBALLS) { /* create_balls(0.003) (env_two_balls_balance_v0.py:212-235) */
                double u[4], pd[3] = {pose.x, pose.y, pose.z}, b1[3], b2[3];
                for (int k = 0; k < 4; k++) u[k] = io.dr.next();
                ugg_tb_balls(pd, UG_TB_BALL_R, u, b1, b2);
                place_object(e, 1, V(b1[0], b1[1], b1[2]), e.obj[0].quat);
                place_object(e, 2, V(b2[0], b2[1], b2[2]), e.obj[0].quat);
            } else {
                v3 bp = V(pose.x, pose.y, pose.z + 0.2 + UG_BB_BALL_R);
                bp.x += io.dr.uniform(-0.03, 0.03);
                bp.y += io.dr.uniform(-0.08, 0.02);
                place_object(e, 1, bp, e.obj[0].quat);
            }
            close_gripper(e, 100.0);
            *next = G_RESET_DONE;
            return L_WAIT;
        }
        case G_RESET_DONE:
            e.goal_approached = 0.0;
            e.goal_grasped = 0.0;
            e.spare = 0.0;
            if (!state_finite(s, e)) { /* a reset that settled into a non-finite state: surfaced (oracle reset_impl) */
                g_sh.flags |= UG_FLAG_NONFINITE;
                g_sh.stats[UG_STAT_NONFINITE]++;
            }
            task_obs(s, e, io.obs);
            io.reset_done = 1;
            *next = G_END;
            return L_NONE;
    }
    *next = G_END;
    return L_NONE;
}
/* wave-wide state_finite(): lane l < NB tests q / qd of dof l, lane NB + j the j-th value of the objects' block
 * (active objects only); one ballot */
__device__ __forceinline__ static int team_nonfinite(const Scene* s) {
    const EnvState& e = g_sh.e;
    const int lane = threadIdx.x;
    bool bad = false;
    if (lane < NB) bad = !__builtin_isfinite(e.q[lane]) || !__builtin_isfinite(e.qd[lane]);
    const int j = lane - NB;
    if (j >= 0 && j < MAXOBJ * UG_OBJ_DOUBLES) {
        const int o = j / UG_OBJ_DOUBLES;
        bad = o < s->nobj && e.oactive[o] != 0.0 && !__builtin_isfinite((&e.obj[0].pos.x)[j]);
    }
    return ballot(bad) != 0ull;
}
/* the non-finite guard voids a runaway state (oracle poison): q, qd and the active objects' state NaN, no contacts */
__device__ __forceinline__ static void team_poison(const Scene* s) {
    EnvState& e = g_sh.e;
    const int lane = threadIdx.x;
    if (lane < NB) { e.q[lane] = __builtin_nan(""); e.qd[lane] = __builtin_nan(""); }
    const int j = lane - NB;
    if (j >= 0 && j < MAXOBJ * UG_OBJ_DOUBLES) {
        const int o = j / UG_OBJ_DOUBLES;
        if (o < s->nobj && e.oactive[o] != 0.0) (&e.obj[0].pos.x)[j] = __builtin_nan("");
    }
    if (lane == 0) e.nman = 0.0;
    __syncthreads();
}
/* runs the program from pc0 to the end; returns physics substeps taken */
__device__ __forceinline__ static int team_run(const Scene* s, double* ws, int pc0, RunIO& io) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    int pc = pc0, ns = 0;
    while (true) {
        PROF_T0(t_glue);
        if (lane == 0) {
            int next;
            sh.is[1] = glue(s, pc, io, &next);
            sh.is[2] = next;
            sh.qsvalid = 0; /* the glue may move, create or remove bodies: the next substep collides in full */
        }
        __syncthreads();
        PROF_ADD(PF_GLUE, t_glue);
        int loop = uniform(sh.is[1]);
        pc = uniform(sh.is[2]);
        if (loop == L_NONE) {
            if (pc == G_END) break;
            continue;
        }
        /* physics: 10 fixed substeps, or wait_until_stable (<= 480 substeps until sum|dq| < eps) */
        double pos = lane < NB ? sh.e.q[lane] : 0.0;
        for (int i = 0;; i++) {
            team_substep(s, ws);
            ns++;
            /* a non-finite state ends the loop at once (oracle wait_until_stable / robot_reset) */
            if (team_nonfinite(s)) {
                team_poison(s);
                break;
            }
            if (loop == L_FIXED10 || loop == L_FIXED120) { /* robot.reset's 10 substeps / Box's 120 per step */
                if (i + 1 == (loop == L_FIXED10 ? 10 : UG_BX_STEPS)) break;
                continue;
            }
            double qn = lane < NB ? sh.e.q[lane] : 0.0;
            if (lane < NB) sh.a12[lane] = ug_fabs(pos - qn);
            __syncthreads();
            if (lane == 0) sh.is[0] = np_sum12(sh.a12) < UG_STABLE_EPS;
            __syncthreads();
            const int stable = uniform(sh.is[0]);
            if (stable || i + 1 == UG_STABLE_STEPS) {
                /* "did not stabilize" (env_ball_balance_v0.py:102-103): surfaced as a flag and a counter */
                if (!stable && lane == 0) { sh.stats[UG_STAT_UNSTABLE]++; sh.flags |= UG_FLAG_UNSTABLE; }
                break;
            }
            pos = qn;
        }
    }
    return ns;
}

/* ---------------- state in/out (cooperative, canonical layout) ---------------- */
__device__ static void team_load(const double* S, const int* stats) {
    Shared& sh = g_sh;
    double* dst = (double*)&sh.e;
    for (int i = threadIdx.x; i < UG_STATE_DIM; i += TEAM) dst[i] = S[i];
    if (threadIdx.x < UG_NSTAT) sh.stats[threadIdx.x] = stats ? stats[threadIdx.x] : 0;
    if (threadIdx.x == 0) { sh.flags = 0; sh.qsvalid = 0; }
    if (threadIdx.x < NB) {
        int m = 0;
        for (int b = threadIdx.x; b >= 0; b = UG_BODY_PARENT[b]) m |= 1 << b;
        sh.anc[threadIdx.x] = m;
        sh.bdepth[threadIdx.x] = body_depth(threadIdx.x);
    }
#ifdef UG_PROF
    for (int i = threadIdx.x; i < UG_NPROF; i += TEAM) sh.prof[i] = 0;
#endif
    __syncthreads();
}
__device__ static void team_prof_flush() {
    Shared& sh = g_sh;
#ifdef UG_PROF
    __syncthreads();
    for (int i = threadIdx.x; i < UG_NPROF; i += TEAM) atomicAdd(&g_prof[i], sh.prof[i]);
#endif
}
/* BallBalance / TwoBalls reset predictor inputs (scheduling only): ball o in the paddle frame -> its paddle-frame
 * offset, velocities and in-plane gravity and the log times of an edge-roll + free-fall estimate (14 inputs,
 * tools/fit_priority.py features()) */
#define UG_BALL_IN 14
__device__ static void bb_ball_inputs(const EnvState& e, const m3& R, int o, double* x) {
    const v3 l = mtv(R, vsub(e.obj[o].pos, e.obj[0].pos));
    const v3 lv = mtv(R, vsub(e.obj[o].v, e.obj[0].v));
    const v3 gl = mtv(R, V(0.0, 0.0, -9.81));
    const double sx = l.x < 0.0 ? -1.0 : (l.x > 0.0 ? 1.0 : 0.0), sy = l.y < 0.0 ? -1.0 : (l.y > 0.0 ? 1.0 : 0.0);
    const double fx = fabs(l.x) / UG_BB_PADDLE_HX, fy = fabs(l.y) / UG_BB_PADDLE_HY;
    const double vx = lv.x * sx, vy = lv.y * sy;
    const double dz = e.obj[o].pos.z - e.obj[0].pos.z, bvz = e.obj[o].v.z;
    const double tf = dz < 0.0 ? 0.0 : (bvz + sqrt(bvz * bvz + 2.0 * 9.81 * dz)) / 9.81;
    const double tex = fx >= 1.0 ? 0.0 : (1.0 - fx) * UG_BB_PADDLE_HX / fmax(vx, 0.05);
    const double tey = fy >= 1.0 ? 0.0 : (1.0 - fy) * UG_BB_PADDLE_HY / fmax(vy, 0.05);
    const double v[UG_BALL_IN] = {fx, fy, l.z, vx, vy, lv.z, dz, bvz, gl.x * sx, gl.y * sy,
                                log(fmin(tex, tey) + tf + 1e-3), log(tex + 1e-3), log(tey + 1e-3), log(tf + 1e-3)};
    for (int i = 0; i < UG_BALL_IN; i++) x[i] = v[i];
}
/* a 1-hidden-layer ReLU MLP's logit over standardised inputs */
template <int IN, int HID>
__device__ static double mlp_logit(const double* x, const double* mu, const double* sd, const double* W1,
                                   const double* B1, const double* W2, double b2) {
    double z[IN];
    for (int i = 0; i < IN; i++) z[i] = (x[i] - mu[i]) / sd[i];
    double out = b2;
    for (int h = 0; h < HID; h++) {
        double a = B1[h];
        for (int i = 0; i < IN; i++) a += z[i] * W1[i * HID + h];
        out += fmax(a, 0.0) * W2[h];
    }
    return out;
}
/* BallBalance: the logit of "this env ends its episode in the next env-step" from the ball's 14 inputs and the step's
 * action, a 17 -> 16 (ReLU) -> 1 MLP (prio_model.h, tools/fit_priority.py; the env leaves the 14 in its k_prio record,
 * k_prio adds the action: held-out misses 0.45 -> 0 of ~264 resets per step) */
static_assert(UG_PM_IN == UG_BALL_IN + 3, "the ball's inputs, the action");
/* TwoBallsBalance: one model over both balls' inputs, the episode's elapsed steps, the paddle's vertical velocity and
 * the next step's action, 34 -> 32 (ReLU) -> 1 (prio_model_tb.h, tools/fit_priority.py --task 6): the larger of two
 * single-ball logits ranked the resets where both balls hit the paddle together last (~55 per step, the launch 37 ms
 * against 23.5 ms for the longest-first order); without the action ~58 of ~420 resets per step ranked outside the
 * first 1024 launch slots, with it ~15.  The env writes its 31 state inputs here (UG_PF_STRIDE doubles per env, the
 * last one a "model applies" flag); k_prio adds the action once it is known and sets the launch level. */
#define UG_PF_STRIDE 32
#define UG_PT_STATE_IN (2 * UG_BALL_IN + 3)
static_assert(UG_PT_IN == UG_PT_STATE_IN + 3, "two balls' inputs, elapsed (clipped, log), the paddle's vz, the action");
static_assert(UG_PT_STATE_IN < UG_PF_STRIDE, "the flag follows the state inputs");
__device__ static void tb_state_inputs(const EnvState& e, const m3& R, int el, double* x) {
    for (int o = 1; o <= 2; o++) bb_ball_inputs(e, R, o, x + (o - 1) * UG_BALL_IN);
    x[2 * UG_BALL_IN] = fmin((double)el, 10.0);
    x[2 * UG_BALL_IN + 1] = log((double)el + 1.0);
    x[2 * UG_BALL_IN + 2] = e.obj[0].v.z;
}
/* Launch-order priority of an env for the next k_step (0..255, higher runs first).  The launch time is the
 * longest env chain, and an env-step that ends its episode carries a ~170-substep autoreset: envs likely
 * to end next step are dispatched first so their reset overlaps the other envs' steps.  Scheduling only --
 * every env computes the same thing whatever its position in the launch.  Predicted truncation: 255;
 * TwoBalls: its own two-ball model in 255 levels (k_prio, with the action); CubesPush(Diff): a step-length model
 * (k_prio, with the action); BallBalance: the reset predictor's logit in 255 levels (k_prio, with the action)
 * (held-out random-action BallBalance x 4096:
 * 0.44 of ~270 resets per step ranked outside the first 1024 launch slots, against 1.1 for an edge-roll +
 * free-fall time and 5.8 for a position-extrapolation score); otherwise the env's last substep count. */
__device__ static int logit_level(double lg, double l0, double dl) {
    const double b = floor((lg - l0) / dl);
    return b > 254.0 ? 254 : (b < 0.0 ? 0 : (int)b); /* a NaN logit: level 0 */
}
/* CubesPush / CubesPushDiff: log(substeps) of the step from the arm's q, qd and the step's action, 27 -> 32 (ReLU) -> 1
 * (prio_model_cp.h, tools/fit_priority.py --task 1): the launch is its longest env (45 ms against 16.8 ms balanced and
 * 39.6 ms longest-first) and the last substep count does not predict it (correlation 0.02; the model 0.82) */
static_assert(UG_PC_IN == 2 * 12 + 3, "q[12], qd[12], the action");
/* CubesGrasp: the logit of "this step runs >= 450 substeps" from q, qd, the step's motor targets minus q, the branch its
 * random.choices takes and a predicted truncation, 33 -> 32 (ReLU) -> 1 (prio_model_cg.h, tools/fit_priority.py --task
 * 2; held-out list schedule 1.22x -> 1.18x of the balanced work, longest-first 1.02x): the branch is
 * drawn in the step itself (env_cubes_grasp_v0.py:127-130) but it is a function of the env's MT19937 stream and the
 * action, both known before the launch -- k_prio peeks the stream's next random() (mt_peek_random, nothing consumed)
 * and evaluates ugg_cg_choose as the glue will.  The env leaves q, qd and its 7 motor targets here; the flag is 4 (5: the
 * step truncates, so its autoreset follows) */
static_assert(UG_PG_IN == 2 * 12 + 7 + 2, "q[12], qd[12], targets - q [7], the branch, the truncation");
/* Golf: the log-odds of "this step runs >= 60 substeps" from q, qd, the ball's position and the step's action, a
 * gradient-boosted tree ensemble (prio_model_gf.h, tools/fit_priority.py --task 3: held-out list schedule 351 -> 300
 * substeps on 512 slots, longest-first 286; an MLP on the same inputs does not separate the long steps).  The env leaves
 * q, qd and the ball's position here; the flag is 6 */
static_assert(UG_PF_GF_IN == 2 * 12 + 3 + 3, "q[12], qd[12], the ball's position, the action");
static_assert(UG_PF_GJ_IN == 2 * 12 + 3 + 6, "GolfJoints: q[12], qd[12], the ball's position, the 6 joint deltas");
__device__ static int team_priority(const Scene* s, int nsub, int el_next, int max_steps, int autoreset, double* pf) {
    const EnvState& e = g_sh.e;
    if (pf) pf[UG_PF_STRIDE - 1] = 0.0; /* k_prio keeps this level unless the TwoBalls model applies */
    const bool trunc_next = autoreset && max_steps > 0 && el_next >= max_steps;
    if constexpr (NB == 12) {
        if (s->task == UG_TASK_CUBESGRASP && pf) {
            for (int j = 0; j < NB; j++) { pf[j] = e.q[j]; pf[NB + j] = e.qd[j]; }
            for (int m = 0; m < 7; m++) pf[2 * NB + m] = e.mtarget[m];
            pf[UG_PF_STRIDE - 1] = trunc_next ? 5.0 : 4.0;
            return trunc_next ? 255 : 0;
        }
    }
    if (trunc_next) return 255;
    if (s->variant == UG_TASK_TWOBALLS && pf && e.oactive[0] != 0.0 && e.oactive[1] != 0.0 && e.oactive[2] != 0.0) {
        tb_state_inputs(e, qmat(e.obj[0].quat), el_next - 1, pf);
        pf[UG_PF_STRIDE - 1] = 1.0;
        return 0;
    }
    if constexpr (NB == 12) { /* Golf (not GolfJoints): the step's length class from q, qd, the ball and (k_prio) the action */
        if ((s->variant == UG_TASK_GOLF || s->variant == UG_TASK_GOLFJOINTS) && pf && e.oactive[1] != 0.0) {
            for (int j = 0; j < NB; j++) { pf[j] = e.q[j]; pf[NB + j] = e.qd[j]; }
            pf[2 * NB] = e.obj[1].pos.x; pf[2 * NB + 1] = e.obj[1].pos.y; pf[2 * NB + 2] = e.obj[1].pos.z;
            pf[UG_PF_STRIDE - 1] = s->variant == UG_TASK_GOLF ? 6.0 : 7.0; /* GolfJoints: its own trees (6 joint deltas) */
            return 0;
        }
    }
    if constexpr (NB == 12) { /* CubesPush / CubesPushDiff: the step's length from q, qd and (k_prio) the action */
        if (s->task == UG_TASK_CUBESPUSH && pf) {
            for (int j = 0; j < NB; j++) { pf[j] = e.q[j]; pf[NB + j] = e.qd[j]; }
            pf[UG_PF_STRIDE - 1] = 2.0;
            return 0;
        }
    }
    if (s->variant == UG_TASK_BALLBALANCE && pf && e.oactive[0] != 0.0 && e.oactive[1] != 0.0) {
        bb_ball_inputs(e, qmat(e.obj[0].quat), 1, pf);
        pf[UG_PF_STRIDE - 1] = 3.0;
        return 0;
    }
    int b = 0;
    while (b < 14 && (2 << b) <= nsub) b++;
    return b;
}
/* manifold slots beyond nman are written as (pair -1, zeros), as ugo_get_state does */
__device__ static void team_store(double* S, int* stats, uint8_t* flags) {
    const Shared& sh = g_sh;
    __syncthreads();
    if (stats && threadIdx.x < UG_NSTAT) stats[threadIdx.x] = sh.stats[threadIdx.x];
    if (flags && threadIdx.x == 0) *flags = (uint8_t)sh.flags;
    const double* src = (const double*)&sh.e;
    int nm = (int)sh.e.nman;
    for (int i = threadIdx.x; i < UG_STATE_DIM; i += TEAM) {
        double v = src[i];
        if (i >= UG_F_MAN && i < UG_F_TASK) {
            int m = (i - UG_F_MAN) / UG_MAN_DOUBLES, f = (i - UG_F_MAN) % UG_MAN_DOUBLES;
            if (m >= nm) v = f == 0 ? -1.0 : 0.0;
        }
        S[i] = v;
    }
}
