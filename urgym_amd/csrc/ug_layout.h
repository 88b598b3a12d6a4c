/* ug_layout.h -- per-environment state layout of the MI355X simulator.
 *
 * Device memory holds one contiguous record of UG_STATE_DIM doubles per env
 * (array-of-structs): the wavefront that owns env i copies state[i * DIM ..]
 * into LDS with 64-lane coalesced loads at kernel start and back at the end.
 * urgym_get_state / urgym_set_state exchange exactly these records -- the
 * canonical layout also used by the CPU restatement's ugo_get_state, so parity
 * tests compare states directly.
 */
#ifndef UG_LAYOUT_H
#define UG_LAYOUT_H

#define UG_MAXOBJ 3          /* paddle + 2 balls (TwoBallsBalance-v0); other tasks use 1-2 */
#define UG_MAXMAN 16
#define UG_PT_DOUBLES 13
#define UG_MAN_DOUBLES (2 + 4 * UG_PT_DOUBLES)

/* field offsets (doubles) */
#define UG_F_Q 0
#define UG_F_QD 12
#define UG_F_MTARGET 24
#define UG_F_MON 31
#define UG_F_OACTIVE 38
#define UG_F_OBJ (UG_F_OACTIVE + UG_MAXOBJ)   /* per object: pos3 quat4 v3 w3 */
#define UG_OBJ_DOUBLES 13
#define UG_F_NMAN (UG_F_OBJ + UG_MAXOBJ * UG_OBJ_DOUBLES)
#define UG_F_MAN (UG_F_NMAN + 1)   /* per manifold: pair, npts, 4 x (lpA3 lpB3 n3 dist imp imp1 imp2) */
#define UG_F_TASK (UG_F_MAN + UG_MAXMAN * UG_MAN_DOUBLES)   /* approached, grasped, overflow (dropped contacts), spare */
/* the poses of the last substep's narrowphase (q, then per object pos3 quat4), taken before that substep's
 * integration: the manifold points' world positions as Bullet reports them (m_positionWorldOnA/B, set by
 * refreshContactPoints at narrowphase time) are their local anchors under these poses (urgym_contact_points) */
#define UG_F_PREV (UG_F_TASK + 4)
#define UG_PREV_DOUBLES (12 + 7 * UG_MAXOBJ)
#define UG_STATE_DIM (UG_F_PREV + UG_PREV_DOUBLES)

/* per-env event counters (urgym_get_stats / ugo_get_stats), cumulative over the handle's life */
#define UG_STAT_UNSTABLE 0   /* wait_until_stable loops that hit 480 substeps without settling (env_*:102-103) */
#define UG_STAT_SPLIT 1      /* substeps whose solve ran the split-impulse (deep penetration) pass */
#define UG_STAT_ROWCAP 2     /* substeps whose contact points exceeded the row capacity (points dropped) */
#define UG_STAT_MANCAP 3     /* substeps whose manifolds exceeded the manifold capacity (manifolds dropped) */
#define UG_STAT_NONFINITE 4  /* env-steps ended by the non-finite state guard */
#define UG_STAT_SUBSTEPS 5   /* physics substeps run */
#define UG_NSTAT 8
/* per-env flags of the last step / reset call (urgym_get_flags; bit set = happened in that call, its same-step
 * autoreset included) */
#define UG_FLAG_UNSTABLE 1   /* a wait_until_stable loop did not settle ("did not stabilize" warning) */
#define UG_FLAG_NONFINITE 2  /* the state became non-finite: the env was terminated (and reset by autoreset) */
#define UG_FLAG_DROPPED 4    /* contacts were dropped at a capacity limit */

/* creation flags (urgym_create_ex / ugo_create_ex).  The default geometry is the full one: the robot's mesh colliders
 * are PyBullet's convex hulls of all mesh vertices (optimizeConvexHull) and the Golf club's disc a true cylinder.
 * UG_GEOM_LOD selects the collision LOD instead (<= 48-vertex hulls, a 16-gon disc prism): faster, knowingly off the
 * reference's geometry. */
#define UG_GEOM_FULL 1       /* the full geometry, explicitly (the default) */
#define UG_GEOM_LOD 2        /* the collision LOD */
#define UG_GEOM_IS_FULL(flags) (((flags) & UG_GEOM_LOD) == 0)
/* contact generation.  The default (neither bit, or UG_CONTACT_GJK) is Bullet's own convex-convex path, the one
 * PyBullet takes for the robot's mesh hulls (btConvexConvexAlgorithm: GJK + EPA, one new point per pair and substep
 * into the persistent manifold).  UG_CONTACT_VIH keeps rounds 1-3's vertex-in-hull generator
 * (up to 4 points per pair and substep from hull vertices against face planes). */
#define UG_CONTACT_GJK 4
#define UG_CONTACT_VIH 8
#define UG_CONTACT_IS_GJK(flags) (((flags) & UG_CONTACT_VIH) == 0)

#define UG_MT_WORDS 625      /* MT19937 state (624) + index, uint32, contiguous per env */

#endif
