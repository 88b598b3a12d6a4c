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

#define UG_MT_WORDS 625      /* MT19937 state (624) + index, uint32, contiguous per env */

#endif
