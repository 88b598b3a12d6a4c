"""Per-env state record layout (urgym_amd/csrc/ug_layout.h, the single source): field offsets in doubles of the
records urgym_get_state / urgym_set_state exchange, evaluated from the header's #defines."""
import os
import re

_HDR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "ug_layout.h")


def _load():
    env = {}
    for m in re.finditer(r"^#define[ \t]+(UG_\w+)[ \t]+(.+?)[ \t]*(?:/\*.*)?$", open(_HDR).read(), re.M):
        name, expr = m.group(1), m.group(2)
        try:
            env[name] = int(eval(expr, {}, dict(env)))
        except Exception:
            pass
    return env


_L = _load()
MAXOBJ = _L["UG_MAXOBJ"]
MAXMAN = _L["UG_MAXMAN"]
F_Q, F_QD, F_MTARGET, F_MON = _L["UG_F_Q"], _L["UG_F_QD"], _L["UG_F_MTARGET"], _L["UG_F_MON"]
F_OACTIVE, F_OBJ, OBJ_DOUBLES = _L["UG_F_OACTIVE"], _L["UG_F_OBJ"], _L["UG_OBJ_DOUBLES"]
F_NMAN, F_MAN, MAN_DOUBLES, PT_DOUBLES = _L["UG_F_NMAN"], _L["UG_F_MAN"], _L["UG_MAN_DOUBLES"], _L["UG_PT_DOUBLES"]
F_TASK, STATE_DIM = _L["UG_F_TASK"], _L["UG_STATE_DIM"]
F_PREV = _L["UG_F_PREV"]  # the last narrowphase's poses: q (12), then per object pos3 quat4
MT_WORDS = _L["UG_MT_WORDS"]


def obj(o):
    """offset of object o's (pos3, quat4, v3, w3)"""
    return F_OBJ + OBJ_DOUBLES * o
