/*
 * crowdnav_state.h — the engine's per-environment state, struct-of-arrays in one HBM blob.
 *
 * One X-macro list is the single source of truth for the blob layout. It is used by
 *   - the HIP engine (crowdnav_dsrnn_amd/csrc/cn_engine.hip)         — device copy,
 *   - the CPU oracle (oracle/cpu_ref.c, test infrastructure only)     — host copy,
 *   - the Python host side (via cn_state_field_info)                  — get/set_state views.
 * so a state captured from one side can be loaded into the other (teacher-forced parity tests,
 * checkpoint/resume of rollouts).
 *
 * Each field is an array; element (env e, slot k) lives at  base + offset(field) + (e*count + k)*sizeof(T).
 * `count` is one of:
 *   CN_CNT_ENV   1            per-env scalar              (robot, episode bookkeeping)
 *   CN_CNT_HUM   N            one per human               (human i of env e at e*N + i: lanes of one env are adjacent)
 *   CN_CNT_PERM  N*(M+1)      RVO2 kd-tree agent order per human simulator, only when M+1 > 10 (else 0)
 *   CN_CNT_MT    624          numpy legacy MT19937 key words
 * Every field array starts on a 256-byte boundary.
 *
 * Reference meaning of each field (paths relative to the CrowdNav_DSRNN checkout):
 *   r_*        Robot agent      crowd_sim/envs/utils/agent.py:27-34 (px,py,gx,gy,vx,vy,theta), radius/v_pref :18-19
 *   r_dv       CrowdSimDict.desiredVelocity[0]  crowd_sim/envs/crowd_sim_dict.py:22,141,212-216 (float32 value)
 *   potential  CrowdSim.potential    crowd_sim/envs/crowd_sim.py:1065-1067, crowd_sim_dict.py:194-198
 *   gtime      CrowdSim.global_time  crowd_sim_dict.py:139,253
 *   last_a*    CrowdSim.last_acceleration   crowd_sim.py:208,1004-1009 (float32 values)
 *   h_*        Human agents     agent.py:27-34 (+ radius, v_pref)
 *   b_*        CrowdSim.last_human_states (robot belief)  crowd_sim.py:199,429-455
 *   o_r/o_vmax/o_dmask   RVO2 simulator parameters frozen at the first ORCA.predict of the episode
 *              crowd_nav/policy/orca.py:91-109 (radius+0.01+safety_space, maxSpeed=v_pref, dummy slots)
 *   o_perm     RVO2 KdTree::agents_ order, which persists across doStep calls of one simulator
 *   ep_*       baselines bench.Monitor episode accumulators (consumed at train.py:266-267)
 *   case_counter  CrowdSim.case_counter[phase]   crowd_sim_dict.py:136-164
 *   mt, mt_pos numpy RandomState (legacy MT19937) global stream, reseeded at every reset
 *              crowd_sim_dict.py:154. CN_RNG_PHILOX: mt[0] = the episode's Philox key word, mt_pos =
 *              words consumed since the reset (the other 623 words are unused)
 */
#ifndef CROWDNAV_STATE_H
#define CROWDNAV_STATE_H

#include <stdint.h>

enum { CN_CNT_ENV = 0, CN_CNT_HUM = 1, CN_CNT_PERM = 2, CN_CNT_MT = 3 };
enum { CN_T_F64 = 0, CN_T_F32 = 1, CN_T_I64 = 2, CN_T_I32 = 3, CN_T_U32 = 4, CN_T_U8 = 5 };

#define CN_MT_N 624

/* X(name, ctype, type_code, count_kind) */
#define CN_STATE_FIELDS(X)                                  \
    X(r_px, double, CN_T_F64, CN_CNT_ENV)                   \
    X(r_py, double, CN_T_F64, CN_CNT_ENV)                   \
    X(r_gx, double, CN_T_F64, CN_CNT_ENV)                   \
    X(r_gy, double, CN_T_F64, CN_CNT_ENV)                   \
    X(r_vx, double, CN_T_F64, CN_CNT_ENV)                   \
    X(r_vy, double, CN_T_F64, CN_CNT_ENV)                   \
    X(r_theta, double, CN_T_F64, CN_CNT_ENV)                \
    X(r_dv, double, CN_T_F64, CN_CNT_ENV)                   \
    X(r_radius, double, CN_T_F64, CN_CNT_ENV)               \
    X(r_vpref, double, CN_T_F64, CN_CNT_ENV)                \
    X(potential, double, CN_T_F64, CN_CNT_ENV)              \
    X(gtime, double, CN_T_F64, CN_CNT_ENV)                  \
    X(last_ax, double, CN_T_F64, CN_CNT_ENV)                \
    X(last_ay, double, CN_T_F64, CN_CNT_ENV)                \
    X(ep_return, double, CN_T_F64, CN_CNT_ENV)              \
    X(case_counter, int64_t, CN_T_I64, CN_CNT_ENV)          \
    X(ep_len, int32_t, CN_T_I32, CN_CNT_ENV)                \
    X(scenario, int32_t, CN_T_I32, CN_CNT_ENV)              \
    X(reset_count, int32_t, CN_T_I32, CN_CNT_ENV)           \
    X(flags, uint32_t, CN_T_U32, CN_CNT_ENV)                \
    X(overflow, uint32_t, CN_T_U32, CN_CNT_ENV)             \
    X(mt_pos, int32_t, CN_T_I32, CN_CNT_ENV)                \
    X(h_px, double, CN_T_F64, CN_CNT_HUM)                   \
    X(h_py, double, CN_T_F64, CN_CNT_HUM)                   \
    X(h_gx, double, CN_T_F64, CN_CNT_HUM)                   \
    X(h_gy, double, CN_T_F64, CN_CNT_HUM)                   \
    X(h_vx, double, CN_T_F64, CN_CNT_HUM)                   \
    X(h_vy, double, CN_T_F64, CN_CNT_HUM)                   \
    X(h_r, double, CN_T_F64, CN_CNT_HUM)                    \
    X(h_vpref, double, CN_T_F64, CN_CNT_HUM)                \
    X(h_theta, double, CN_T_F64, CN_CNT_HUM)                \
    X(b_px, double, CN_T_F64, CN_CNT_HUM)                   \
    X(b_py, double, CN_T_F64, CN_CNT_HUM)                   \
    X(b_vx, double, CN_T_F64, CN_CNT_HUM)                   \
    X(b_vy, double, CN_T_F64, CN_CNT_HUM)                   \
    X(b_r, double, CN_T_F64, CN_CNT_HUM)                    \
    X(o_r, float, CN_T_F32, CN_CNT_HUM)                     \
    X(o_vmax, float, CN_T_F32, CN_CNT_HUM)                  \
    X(o_dmask, uint32_t, CN_T_U32, CN_CNT_HUM)              \
    X(o_perm, uint8_t, CN_T_U8, CN_CNT_PERM)                \
    X(mt, uint32_t, CN_T_U32, CN_CNT_MT)

/* flags bits (per env) */
#define CN_FLAG_ORCA_FROZEN 0x1u  /* RVO2 simulators of this episode exist (first predict happened) */
#define CN_FLAG_NAN 0x2u          /* a NaN/Inf appeared in the state (e.g. social force at goal) */
#define CN_FLAG_ROBOT_F32 0x4u    /* robot vx/vy (and unicycle theta) now hold numpy float32 values: the
                                     reference's robot state is int/python-float at reset and becomes
                                     np.float32 after the first step (NEP 50 promotion), which moves its
                                     heading/trig to float32 (agent.py:186-212, crowd_sim.py:821-833) */

enum {
#define CN_X_ENUM(name, ctype, tcode, cnt) CN_F_##name,
    CN_STATE_FIELDS(CN_X_ENUM)
#undef CN_X_ENUM
    CN_NUM_FIELDS
};

/* Number of agents in one human's RVO2 simulator: self + (N-1) humans (+ robot if visible). */
static inline int cn_sim_agents(int N, int robot_visible) { return N + (robot_visible ? 1 : 0); }

/* Elements per env of a field kind. */
static inline int64_t cn_count_of(int kind, int N, int robot_visible)
{
    int A = cn_sim_agents(N, robot_visible);
    switch (kind) {
    case CN_CNT_ENV: return 1;
    case CN_CNT_HUM: return N;
    case CN_CNT_PERM: return A > 10 ? (int64_t)N * A : 0;
    default: return CN_MT_N;
    }
}

static inline int64_t cn_type_size(int tcode)
{
    switch (tcode) {
    case CN_T_F64: case CN_T_I64: return 8;
    case CN_T_F32: case CN_T_I32: case CN_T_U32: return 4;
    default: return 1;
    }
}

/* Fill offsets[CN_NUM_FIELDS] (bytes from blob start); return total blob bytes. */
static inline int64_t cn_state_layout(int64_t E, int N, int robot_visible, int64_t *offsets)
{
    static const int kinds[] = {
#define CN_X_KIND(name, ctype, tcode, cnt) cnt,
        CN_STATE_FIELDS(CN_X_KIND)
#undef CN_X_KIND
    };
    static const int tcodes[] = {
#define CN_X_T(name, ctype, tcode, cnt) tcode,
        CN_STATE_FIELDS(CN_X_T)
#undef CN_X_T
    };
    int64_t off = 0;
    for (int f = 0; f < CN_NUM_FIELDS; ++f) {
        off = (off + 255) & ~(int64_t)255;
        if (offsets) offsets[f] = off;
        off += E * cn_count_of(kinds[f], N, robot_visible) * cn_type_size(tcodes[f]);
    }
    return (off + 255) & ~(int64_t)255;
}

/* Typed field pointers into a blob (host or device address). */
typedef struct cn_state_ptrs {
#define CN_X_PTR(name, ctype, tcode, cnt) ctype *name;
    CN_STATE_FIELDS(CN_X_PTR)
#undef CN_X_PTR
} cn_state_ptrs;

static inline void cn_state_bind(cn_state_ptrs *p, void *blob, int64_t E, int N, int robot_visible)
{
    int64_t off[CN_NUM_FIELDS];
    cn_state_layout(E, N, robot_visible, off);
    char *b = (char *)blob;
#define CN_X_BIND(name, ctype, tcode, cnt) p->name = (ctype *)(b + off[CN_F_##name]);
    CN_STATE_FIELDS(CN_X_BIND)
#undef CN_X_BIND
}

#endif /* CROWDNAV_STATE_H */
