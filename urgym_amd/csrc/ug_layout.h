/* ug_layout.h -- per-environment state layout of the MI355X simulator.
 *
 * Device memory holds every field structure-of-arrays: field f of env i lives
 * at state[f * n_envs + i] (FP64), so a wavefront loading one field touches
 * 64 consecutive doubles (512 B, fully coalesced).  urgym_get_state /
 * urgym_set_state exchange the same fields per env (array-of-structs,
 * UG_STATE_DIM doubles per env) -- the canonical layout also used by the CPU
 * restatement's ugo_get_state, so parity tests compare states directly.
 */
#ifndef UG_LAYOUT_H
#define UG_LAYOUT_H

#define UG_MAXOBJ 2
#define UG_MAXMAN 16
#define UG_PT_DOUBLES 13
#define UG_MAN_DOUBLES (2 + 4 * UG_PT_DOUBLES)

/* field offsets (doubles) */
#define UG_F_Q 0
#define UG_F_QD 12
#define UG_F_MTARGET 24
#define UG_F_MON 31
#define UG_F_OACTIVE 38
#define UG_F_OBJ 40          /* per object: pos3 quat4 v3 w3 */
#define UG_OBJ_DOUBLES 13
#define UG_F_NMAN 66
#define UG_F_MAN 67          /* per manifold: pair, npts, 4 x (lpA3 lpB3 n3 dist imp imp1 imp2) */
#define UG_F_TASK (UG_F_MAN + UG_MAXMAN * UG_MAN_DOUBLES)   /* approached, grasped, overflow, spare */
#define UG_STATE_DIM (UG_F_TASK + 4)

#define UG_MT_WORDS 625      /* MT19937 state (624) + index, uint32 SoA */

#endif
