/*
 * crowdnav.h — C ABI of the MI355X batched CrowdSimDict engine (libcrowdnav_hip.so).
 *
 * Drop-in boundary for the reference's env hot path. Each entry point replaces a reference
 * interface (paths relative to the CrowdNav_DSRNN checkout):
 *
 *   cn_create     ⟵ gym.make('CrowdSimDict-v0') + CrowdSim.configure(config) + make_env's
 *                   thisSeed/nenv/phase assignment, for E envs at once
 *                   (crowd_sim/__init__.py:9-11, crowd_sim/envs/crowd_sim.py:93-246,
 *                    pytorchBaselines/a2c_ppo_acktr/envs.py:46-75)
 *   cn_reset      ⟵ CrowdSimDict.reset() of every env (crowd_sim/envs/crowd_sim_dict.py:105-203),
 *                   i.e. ShmemVecEnv.reset (shmem_vec_env.py:89-95) + VecPyTorch.reset (envs.py:215-222)
 *   cn_step       ⟵ CrowdSimDict.step(action) of every env (crowd_sim_dict.py:205-271) followed by the
 *                   VecEnv worker's auto-reset (shmem_vec_env.py:164-168) and bench.Monitor's episode
 *                   bookkeeping; i.e. VecPyTorch.step (envs.py:224-239) minus the Python info dicts
 *   cn_get_state / cn_set_state   ⟵ no reference equivalent (state lives in forked workers there);
 *                   used for teacher-forced parity tests and rollout checkpointing
 *   cn_edge_features ⟵ the input layers of the DSRNN forward, fused:
 *                   HumanHumanEdgeRNN.encoder_linear+ReLU (srnn_model.py:210-211) for the temporal and
 *                   spatial edges, SRNN.robot_linear (srnn_model.py:466) and
 *                   HumanNodeRNN.encoder_linear+ReLU (srnn_model.py:160-161)
 *   cn_gru_fwd_step / cn_gru_bwd_step ⟵ one time step of the mask-segmented GRU
 *                   (srnn_model.py:52-104 RNNBase._forward_gru, torch nn.GRU cell math) and its gradient;
 *                   cn_gru_fwd_fused runs the recurrent GEMM hm W_hh^T on the f32 MFMA with the gates in its
 *                   epilogue (the forward's per-step kernel); cn_gru_fwd_seq / cn_gru_bwd_seq run whole
 *                   sequences (up to two GRUs per launch; the backward's dgh W_hh on the MFMA with the gate
 *                   gradients in its epilogue); x W_ih^T and the weight gradients over all steps remain
 *                   library GEMMs
 *   cn_gaussian_act ⟵ the act() tail of DiagGaussian / FixedNormal (distributions.py:36-94): sample or
 *                   mode and the summed log-probability
 *   cn_gae         ⟵ RolloutStorage.compute_returns with use_gae (storage.py:132-177), one launch per rollout
 *   cn_orca_predict / cn_orca_predict_kd / cn_social_force_predict ⟵ the agent policy plugin
 *                   policy_factory[name](config).predict(JointState) (crowd_nav/policy/policy_factory.py:1-17)
 *   cn_lidar_obs     ⟵ CrowdSimDict.generate_ob's 'convgru' observation (crowd_sim_dict.py:96-101) with
 *                   LidarSensor.sensor_spin (crowd_sim/envs/utils/lidarv2.py:398-427) evaluated at reset
 *   cn_wgrad       ⟵ the weight / bias gradient of the Linear layers with a tiny side (autograd's dy^T x)
 *   cn_attn_pool_fwd / cn_attn_pool_bwd ⟵ EdgeAttention's weighted sum of the spatial edge states
 *                   (srnn_model.py:320-333, torch.bmm(h_spatials^T, attn)) and its gradient
 *   cn_spatial_attn_fwd / cn_spatial_attn_bwd ⟵ EdgeAttention's whole spatial branch (spatial_edge_layer,
 *                   att_func's scores and softmax, the pooling: srnn_model.py:256-333) in one pass over
 *                   h_spatials, and its gradient (the training and act() paths use these)
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (torch tensors' data_ptr()), row-major, caller-owned.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream). Calls are
 *     stream-ordered and asynchronous; no call allocates or synchronises except cn_create/cn_destroy
 *     and the host-copy variants of get/set_state.
 *   - Every call returns 0 on success or a negative CN_E* code; cn_last_error() gives a message
 *     (thread-local). Unsupported reference options are rejected by cn_create with CN_EUNSUPPORTED.
 */
#ifndef CROWDNAV_H
#define CROWDNAV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes */
#define CN_OK 0
#define CN_EINVAL (-1)
#define CN_EUNSUPPORTED (-2)
#define CN_EHIP (-3)
#define CN_ENOMEM (-4)

/* robot kinematics  (config.action_space.kinematics, crowd_nav/configs/config.py:137) */
#define CN_HOLONOMIC 0
#define CN_UNICYCLE 1
/* human policies    (policy_factory, crowd_nav/policy/policy_factory.py:1-17) */
#define CN_POLICY_ORCA 0
#define CN_POLICY_SOCIAL_FORCE 1
/* phases            (crowd_sim.py:110-119, 690-694) */
#define CN_PHASE_TRAIN 0
#define CN_PHASE_VAL 1
#define CN_PHASE_TEST 2
/* scenarios         (create_agent_attributes, crowd_sim.py:296-357) */
#define CN_SC_CIRCLE_CROSSING 0
#define CN_SC_SQUARE_CROSSING 1
#define CN_SC_PARALLEL_TRAFFIC 2
#define CN_SC_PERPENDICULAR_TRAFFIC 3
#define CN_SC_SIDE_PREF_PASSING 4
#define CN_SC_SIDE_PREF_OVERTAKING 5
#define CN_SC_SIDE_PREF_CROSSING 6
/* scenario selection at reset (crowd_sim_dict.py:110-125) */
#define CN_SCMODE_ROUND_ROBIN 0  /* env g uses scenarios[g % n]; n == 1 is the deterministic reference case */
#define CN_SCMODE_SEQUENTIAL 1   /* test.social_metrics: scenarios[reset_count % n] (crowd_sim_dict.py:114-122) */
/* random stream of resets and goal changes (crowd_sim_dict.py:154 reseeds numpy's global RandomState) */
#define CN_RNG_MT19937 0  /* parity: numpy legacy MT19937 per env, the reference's exact draws */
#define CN_RNG_PHILOX 1   /* fast mode: Philox4x32-10, key (episode seed, 0x43726f77), counter = word / 4;
                             same draw order and distributions, different values; no 2.5 KB key per env */
/* step events (crowd_sim/envs/utils/info.py) */
#define CN_EV_NOTHING 0
#define CN_EV_DANGER 1
#define CN_EV_COLLISION 2
#define CN_EV_REACHGOAL 3
#define CN_EV_TIMEOUT 4

/* per-step info metrics, float32 [E][CN_INFO_K]  (step_info keys, crowd_sim.py:973-1030) */
#define CN_INFO_AGG_NAV_TIME 0
#define CN_INFO_PATH_VIOLATION 1
#define CN_INFO_PERSONAL_VIOLATION 2
#define CN_INFO_JERK_COST 3
#define CN_INFO_DIST_TO_GOAL 4
#define CN_INFO_SPEED_VIOLATION 5
#define CN_INFO_MIN_DIST 6     /* Danger(min_dist) payload; dmin (inf if no human counted) */
#define CN_INFO_SCENARIO 7
#define CN_INFO_SIDE_LEFT 8    /* test.side_preference only (crowd_sim.py:977-992) */
#define CN_INFO_SIDE_RIGHT 9
#define CN_INFO_SEPARATION 10
#define CN_INFO_OVERFLOW 11    /* bounded-rejection overflows so far in this episode (engine diagnostic) */
#define CN_INFO_K 12

#define CN_MAX_SCENARIOS 8

typedef struct cn_config {
    /* batch geometry */
    int32_t num_envs;      /* E: envs owned by this engine instance (one device) */
    int32_t human_num;     /* N: config.sim.human_num */
    int64_t env_offset;    /* global index of local env 0 (sharding); thisSeed = seed + global index */
    int64_t nenv;          /* the reference's env.nenv = num_processes over ALL shards (envs.py:69) */
    int64_t seed;          /* config.env.seed (envs.py:66) */
    int32_t phase;         /* CN_PHASE_*; make_env uses 'train' if nenv > 1 else 'test' (envs.py:70-73) */
    int32_t kinematics;    /* CN_HOLONOMIC / CN_UNICYCLE */
    int32_t human_policy;  /* CN_POLICY_* */
    int32_t scenario_mode; /* CN_SCMODE_* */
    int32_t num_scenarios;
    int32_t scenarios[CN_MAX_SCENARIOS];
    int32_t val_size, test_size;          /* config.env.val_size / test_size (case_size) */
    /* env (config.env / config.sim) */
    double time_step, time_limit, circle_radius, square_width;
    /* agents */
    double robot_radius, robot_vpref, robot_fov; /* fov in radians = pi * config.robot.FOV */
    double human_radius, human_vpref, human_fov;
    int32_t robot_visible, randomize_attributes;
    int32_t random_goal_changing, end_goal_changing, random_radii, random_v_pref;
    double goal_change_chance, end_goal_change_chance;
    /* reward (config.reward) */
    double success_reward, collision_penalty, discomfort_dist, discomfort_penalty_factor;
    double potential_factor, norm_zone_penalty;
    int32_t potential_based, time_factor, norm_zones, norm_zone_lhs;
    /* social (config.social / config.test) */
    double min_personal_space, max_walking_speed;
    int32_t social_metrics, side_preference;
    /* human policies (config.orca / config.sf) */
    double orca_neighbor_dist, orca_safety_space, orca_time_horizon, orca_time_horizon_obst;
    double sf_A, sf_B, sf_KI;
    /* engine */
    int32_t max_tries;     /* bounded rejection sampling (reference loops forever) */
    int32_t rng_mode;      /* CN_RNG_MT19937 (default) / CN_RNG_PHILOX */
} cn_config;

typedef struct cn_engine cn_engine;

const char *cn_last_error(void);
const char *cn_version(void);

int cn_config_validate(const cn_config *cfg);
int cn_create(const cn_config *cfg, int device, cn_engine **out);
void cn_destroy(cn_engine *eng);

/* Mixed engine: per-env scenario dispatch with per-env human counts in ONE engine (the
 * reference picks a scenario per env reset, crowd_sim_dict.py:112-125, and the side-preference scenarios
 * run with their own human count / circle radius / fixed robot, crowd_sim.py:334-357,642-651).
 * Env r (global index env_offset + r) belongs to group env_group[r]; groups[g] is a full cn_config for
 * its envs (num_envs = how many envs env_group assigns to g; env_offset / nenv / seed / phase equal across
 * groups; round-robin scenario mode with the FULL scenario list, so env r's scenario
 * scenarios[(env_offset + r) % num_scenarios] must be one group env_group[r] is configured for).
 * The engine then behaves as one engine of num_envs envs with N = max human_num: cn_reset / cn_step take
 * [num_envs]-row buffers; spatial_edges rows beyond an env's own human count are padding (a never-seen
 * human: belief (15, 15) relative to the robot). cn_step launches one step kernel per group.
 * cn_get_state / cn_set_state: the groups' blobs concatenated in group order; cn_state_device_ptr: NULL;
 * cn_lidar_obs: CN_EUNSUPPORTED. */
int cn_create_mixed(const cn_config *groups, int num_groups, const int32_t *env_group, int64_t num_envs, int device,
                    cn_engine **out);
/* per-env human count, into host memory [E] (a plain engine: N everywhere) */
int cn_env_humans(const cn_engine *eng, int32_t *dst);

/* Reset all envs (fresh episodes, case_counter continues). obs out: robot_node [E][7], temporal [E][2],
 * spatial [E][N][2] float32. */
int cn_reset(cn_engine *eng, void *stream, float *robot_node, float *temporal_edges, float *spatial_edges);

/* One step of every env with auto-reset of finished envs.
 * in : actions [E][2] float32 (raw policy output; clipped in place semantics of SRNN.clip_action are
 *      NOT applied to the caller's buffer — the reference mutates its private numpy copy)
 * out: obs (first obs of the new episode where done), reward [E] f32, done [E] u8, event [E] i8,
 *      info [E][CN_INFO_K] f32, ep_return [E] f64 and ep_len [E] i32 (Monitor 'r'/'l', valid where done).
 * Any output pointer except the obs may be NULL. */
int cn_step(cn_engine *eng, void *stream, const float *actions,
            float *robot_node, float *temporal_edges, float *spatial_edges,
            float *reward, uint8_t *done, int8_t *event, float *info,
            double *ep_return, int32_t *ep_len);

/* T consecutive cn_step calls issued from native code: step t takes actions + t * action_stride
 * (floats; >= 2 * E, e.g. a [T][E][2] tensor), the outputs are those of the last step (each step
 * overwrites them, as T cn_step calls would). For open-loop action sequences (scripted or pre-drawn
 * actions, bench.py's synthetic windows): the launches go back to back without a host round trip per
 * step. Same kernels, same results as the T single calls. */
int cn_step_seq(cn_engine *eng, void *stream, int T, const float *actions, int64_t action_stride,
                float *robot_node, float *temporal_edges, float *spatial_edges,
                float *reward, uint8_t *done, int8_t *event, float *info,
                double *ep_return, int32_t *ep_len);

/* State blob (layout: include/crowdnav_state.h). */
/* Graph mode (on = 1): the step sequence (triple-buffered spawn-list indices, launch ids, the draw-all flag
 * after cn_reset / cn_set_state) moves from the host into device memory, so cn_step launches carry no
 * per-call arguments and a sequence of cn_step calls (with the caller's other work) can be captured once in
 * a hipGraph and replayed (learner RolloutTrainer). Costs the launch's last workgroup one atomic; off by
 * default (separate kernel variants). Plain engines only (CN_EUNSUPPORTED for cn_create_mixed). Switching
 * synchronises `stream`. No reference equivalent (its env steps are host processes). The engine issues no
 * hipMemsetAsync on a stream (graph mode's flag writes are kernels), so a capture never holds a memset node
 * from it: see cn_graph_node_counts. */
int cn_set_graph_mode(cn_engine *eng, void *stream, int on);

/* Node census of a captured hipGraph_t (`graph`): counts[k] = nodes of hipGraphNodeType k for k < n (n <= 32;
 * kernel = 0, memcpy = 1, memset = 2, ...). The rollout trainer refuses to replay a graph that holds memset
 * nodes: on this ROCm runtime a replayed memset node can write stale bytes instead of its value (DESIGN.md §4,
 * "HIP-graph memset nodes"), e.g. torch's multi-block reductions then skip writing their result. Returns the
 * total node count in *total. No reference equivalent. */
int cn_graph_node_counts(void *graph, int64_t *counts, int n, int64_t *total);

int cn_state_bytes(const cn_engine *eng, int64_t *bytes);
int cn_state_layout_offsets(const cn_config *cfg, int64_t *offsets, int64_t *total_bytes);
int cn_state_field_info(int field, const char **name, int *type_code, int *count_kind);
int cn_get_state(cn_engine *eng, void *stream, void *dst, int dst_on_host);
int cn_set_state(cn_engine *eng, void *stream, const void *src, int src_on_host);
const void *cn_state_device_ptr(const cn_engine *eng);

/* Kernel timing (measurement hook for bench.py's roofline): while enabled, cn_step records one HIP event
 * on its stream before the first and one after the `max_steps`-th step launch of the window (per-launch
 * event pairs would cost ~12 us of stream time per step). cn_profile_read synchronises on the closing
 * event and returns the window's span in step_kernel_ms (back-to-back launches: the summed launch
 * durations) and the launch count; rng_kernel_ms is always 0 (the RNG work is fused into the step
 * kernel). Reading an incomplete window is CN_EINVAL. */
int cn_profile(cn_engine *eng, int enable, int max_steps);
int cn_profile_read(cn_engine *eng, double *step_kernel_ms, double *rng_kernel_ms, int64_t *launches);

/* Fused DSRNN edge-feature assembly (SRNN input layers), float32, device pointers.
 *   robot_node [E][7], temporal [E][2], spatial [E][N][2]
 *   Wt [64][2] bt[64]  (humanhumanEdgeRNN_temporal.encoder_linear)
 *   Ws [64][2] bs[64]  (humanhumanEdgeRNN_spatial.encoder_linear)
 *   Wr [3][7]  br[3]   (robot_linear)
 *   Wn [64][3] bn[64]  (humanNodeRNN.encoder_linear)
 * out: temporal_embed [E][64], spatial_embed [E][N][64], node_embed [E][64]  (post-ReLU) */
int cn_edge_features(void *stream, int64_t E, int N,
                     const float *robot_node, const float *temporal_edges, const float *spatial_edges,
                     const float *Wt, const float *bt, const float *Ws, const float *bs,
                     const float *Wr, const float *br, const float *Wn, const float *bn,
                     float *temporal_embed, float *spatial_embed, float *node_embed);

/* One GRU step after the two GEMMs (nn.GRU gate order r | z | n, ATen's cell arithmetic):
 *   r = sigmoid(gh_r + gi_r), z = sigmoid(gh_z + gi_z), n = tanh(gi_n + r * gh_n), h = (hm - n) * z + n
 * gi = x W_ih^T + b_ih, gh = hm W_hh^T + b_hh: [B][3H]; hm: [B][H] (previous state times this step's mask);
 * m_next [B] (next step's mask; NULL = 1); out h_out [B][H]; hm_next [B][H] = h * m_next (NULL = skip);
 * save [B][4H] = r | z | n | gh_n for the backward (NULL = skip). H % 4 == 0. */
int cn_gru_fwd_step(void *stream, int64_t B, int H, const float *gi, const float *gh, const float *hm,
                    const float *m_next, float *h_out, float *hm_next, float *save);
/* cn_gru_fwd_step plus a second copy of the new state h_out, written in a grouped row layout: row b at
 * h_out2 + (b / g2) * ld2 + (b % g2) * H (16-byte aligned, ld2 >= g2 * H, ld2 % 4 == 0). Lets the
 * inference step write the temporal (g2 = 1) and spatial (g2 = N) edge states straight into the
 * reference's (B, N + 1, H) 'human_human_edge_rnn' layout (srnn_model.py:406-407, 450, 460) instead of
 * a torch.cat + copy; h_out2 = NULL is cn_gru_fwd_step. */
int cn_gru_fwd_step_scatter(void *stream, int64_t B, int H, const float *gi, const float *gh, const float *hm,
                         const float *m_next, float *h_out, float *hm_next, float *save, float *h_out2, int64_t g2,
                         int64_t ld2);

/* Fused step: the recurrent GEMM gh = hm W_hh^T + b_hh (w_hh [3H][H] row-major, as nn.GRU's weight_hh_l0;
 * b_hh [3H]) on the f32 matrix cores with cn_gru_fwd_step_scatter's gate epilogue, so gh never leaves the
 * chip. Same outputs and arguments as cn_gru_fwd_step_scatter otherwise; H % 32 == 0; hm, w_hh, gi, b_hh,
 * h_out, hm_next and save 16-byte aligned (float4 accesses) with rows contiguous; CN_EINVAL otherwise. Replaces torch.addmm + cn_gru_fwd_step per time step of
 * srnn_model.py:52-104's nn.GRU. */
int cn_gru_fwd_fused(void *stream, int64_t B, int H, const float *gi, const float *hm, const float *w_hh,
                     const float *b_hh, const float *m_next, float *h_out, float *hm_next, float *save, float *h_out2,
                     int64_t g2, int64_t ld2);

/* Gradient of one step. In: acc [B][H] = dL/dhm of the later step (or dL/dh_T at the last step, with
 * m_next = NULL), m_next [B] that later step's mask, dout [B][H] = dL/dh_t from the outputs (NULL = 0),
 * save / hm as written by the forward. Out: dgi, dgh [B][3H] (pre-activation gradients of gi, gh) and
 * acc <- dL/dh_t * z (the caller then adds dgh W_hh to obtain dL/dhm_t). */
int cn_gru_bwd_step(void *stream, int64_t B, int H, float *acc, const float *m_next, const float *dout,
                    const float *save, const float *hm, float *dgi, float *dgh);
/* cn_gru_bwd_step with the bias gradients folded in: the same dgi_t / dgh_t / acc, plus the column sums of
 * dr | dz | dn | dhn of every 16-row block to part [cn_gru_bias_blocks(B)][4H] (H in {64, 128, 256}); after
 * the last step cn_gru_bias_reduce sums the partials of all steps, part [rows][4H], in a fixed order into
 * db_ih = (dr, dz, dn) and db_hh = (dr, dz, dhn) sums ([3H] each; work: cn_gru_bias_work_elems(H) floats).
 * Replaces the reference autograd's two extra passes over [T][B][3H] (dgi.sum(0), dgh.sum(0)). */
int64_t cn_gru_bias_blocks(int64_t B);
int cn_gru_bwd_step_bias(void *stream, int64_t B, int H, float *acc, const float *m_next, const float *dout,
                         const float *save, const float *hm, float *dgi, float *dgh, float *part);
/* cn_gru_bwd_step_bias with the gate gradients stored once, g [B][4H] = [dn | dr | dz | dhn] per row:
 * dgh_t = g[:, H:4H] and dgi_t = g[:, 0:3H] in gate order (n, r, z) (dgi's r / z columns equal dgh's), 2H
 * fewer floats written per row than the separate dgi / dgh. Same acc and bias partials. */
int cn_gru_bwd_step_gates(void *stream, int64_t B, int H, float *acc, const float *m_next, const float *dout,
                          const float *save, const float *hm, float *g, float *part);
int64_t cn_gru_bias_work_elems(int H);
int cn_gru_bias_reduce(void *stream, int64_t rows, int H, const float *part, float *db_ih, float *db_hh,
                       float *work);

/* The act() tail of the Box-action policy (distributions.py:74-94: DiagGaussian with AddBias(zeros) log-std,
 * FixedNormal.sample / .mode and .log_probs) for E envs in one launch: std = exp(logstd) [A],
 * action = eps * std + mean (eps [E][A] from the caller's N(0, 1) draw) or mean when eps = NULL,
 * logp [E] = sum over the A dims of the Normal log-density of action, in torch's float32 operation order.
 * mean, eps, action: [E][A]; A <= 64. */
int cn_gaussian_act(void *stream, int64_t E, int A, const float *mean, const float *logstd, const float *eps,
                    float *action, float *logp);

/* One step of up to two GRUs of the same H in one launch (the act() path's temporal and spatial edge RNNs,
 * srnn_model.py:455-460 at T = 1): cn_gru_fwd_fused per GRU, with the input projection in the kernel when
 * x is given (gi NULL: x [B][F], w_ih [3H][F], b_ih [3H], F % 32 == 0; every GRU of a call in the same mode)
 * and the optional grouped copy h_out2 (g2, ld2) of cn_gru_fwd_step_scatter. No mask / save outputs. */
typedef struct cn_gru_step_seg {
    int64_t B;
    const float *gi;
    const float *x;
    const float *w_ih;
    const float *b_ih;
    int64_t F;
    const float *hm;     /* [B][H] masked state */
    const float *w_hh;
    const float *b_hh;
    float *h_out;        /* [B][H] */
    float *h_out2;       /* grouped copy or NULL */
    int64_t g2;
    int64_t ld2;
} cn_gru_step_seg;
int cn_gru_fwd_step_group(void *stream, int H, int nseg, const cn_gru_step_seg *segs);

/* Returns by generalized advantage estimation (storage.py:132-177 compute_returns with use_gae), one launch
 * for the whole rollout: rewards [T][E], values / masks / bad_masks [T + 1][E] (values[T] = next_value),
 * returns [T + 1][E] (rows 0 .. T-1 written); the reference's float32 operation order per step, with gamma and
 * gamma_lambda = gamma * gae_lambda as float32 scalars; use_proper_time_limits multiplies by bad_masks. */
int cn_gae(void *stream, int T, int64_t E, float gamma, float gamma_lambda, int use_proper_time_limits,
           const float *rewards, const float *values, const float *masks, const float *bad_masks, float *returns);

/* Whole sequences: the T-step loops of srnn_model.py:52-104's nn.GRU (forward) and of its autograd backward
 * issued from native code, one launch per step for up to two independent GRUs of the same H at once (the
 * DSRNN's spatial and temporal edge RNNs, srnn_model.py:455-460; their rows share each launch). H % 32 == 0;
 * every array 16-byte aligned with rows contiguous; 1 <= nseg <= 2. */
typedef struct cn_gru_seq_fwd {
    int64_t B;           /* rows */
    const float *gi;     /* [T][B][3H] = x W_ih^T + b_ih, or NULL: the kernel projects x itself (below) */
    const float *w_hh;   /* [3H][H] (weight_hh_l0) */
    const float *b_hh;   /* [3H] */
    const float *m;      /* [T][B] masks */
    float *out;          /* [T][B][H] outputs */
    float *hm;           /* [nh][B][H] masked states: hm[0] = h0 * m[0] (caller); step t reads hm[t % nh] and
                            writes hm[(t + 1) % nh] = h_t * m[t + 1] (nh = T keeps all of them for the backward) */
    float *save;         /* [T][B][4H] r | z | n | gh_n per step for the backward, or NULL */
    int64_t nh;          /* 1 <= nh <= T; nh >= 2 when T > 1 (a step's workgroups read hm[t % nh] while others
                            write hm[(t + 1) % nh]); nh == T when save is not NULL (the backward reads every hm) */
    const float *x;      /* [T][B][F] GRU inputs when gi is NULL (then gi is never stored: the step kernel runs */
    const float *w_ih;   /* x W_ih^T on the MFMA ahead of hm W_hh^T); w_ih [3H][F] (weight_ih_l0), b_ih [3H], */
    const float *b_ih;   /* F % 32 == 0. Every GRU of a call uses the same mode. */
    int64_t F;
} cn_gru_seq_fwd;
/* cn_gru_fwd_fused for t = 0 .. T - 1 (same arithmetic per row and step; like cn_gru_fwd_fused, a launch with
 * fewer 128-row tiles than CUs splits K over the workgroup's waves on 32-row tiles). */
int cn_gru_fwd_seq(void *stream, int T, int H, int nseg, const cn_gru_seq_fwd *segs);

typedef struct cn_gru_seq_bwd {
    int64_t B;
    const float *w_hh_t; /* [H][3H] = weight_hh_l0 transposed */
    const float *m;      /* [T][B] masks */
    const float *dout;   /* [T][B][H] dL/d out, or NULL */
    const float *save;   /* [T][B][4H] and */
    const float *hm;     /* [T][B][H] as written by cn_gru_fwd_seq (nh = T) */
    float *acc;          /* [B][H] in: dL/dh_{T-1} through the final state (zeros if unused);
                            out: dL/d hm_0 (the caller multiplies by m[0] for dL/dh0) */
    float *g;            /* [T][B][4H] out: dn | dr | dz | dhn per step (dgh_t = g[t][:, H:4H], dgi_t = g[t][:, 0:3H]
                            in gate order n, r, z) */
    float *db_ih;        /* [3H] out: the bias gradients (sums over all T * B rows, fixed order) */
    float *db_hh;        /* [3H] out */
} cn_gru_seq_bwd;
/* floats of workspace cn_gru_bwd_seq needs for these GRUs (reads only the B fields; the row tiling follows the
 * current device's CU count, so query on the device the backward runs on) */
int64_t cn_gru_bwd_seq_work_elems(int T, int H, int nseg, const cn_gru_seq_bwd *segs);
/* The backward of cn_gru_fwd_seq: T + 1 launches of one fused kernel, each the recurrent GEMM
 * acc_t = a_t + dgh_t W_hh of one step on the f32 matrix cores with the gate gradients of the step before in
 * its epilogue (cn_gru_bwd_step_gates' arithmetic; launches with fewer 128-row tiles than CUs split K over
 * the workgroup's waves on 32-row tiles), then the bias reduction; replaces the per-step
 * cn_gru_bwd_step_gates + GEMM pair. work_elems = the floats at work; fails (CN_EINVAL) when it is below
 * cn_gru_bwd_seq_work_elems on the current device. */
int cn_gru_bwd_seq(void *stream, int T, int H, int nseg, const cn_gru_seq_bwd *segs, float *work, int64_t work_elems);

/* The ConvGRU observation row of every env, obs [E][7 + beams] float32:
 *   [clip(robot (px, py, radius, gx, gy, v_pref, theta) / max_range, 0, 1), scan].
 * lidar [E][beams] (caller-owned, zero-initialised) holds each env's current scan
 * |1 - clip(dist / max_range, 0, 1)|. For envs with reset_mask[e] != 0 (NULL = all envs, i.e. after
 * cn_reset; pass the `done` output of cn_step after a step) the observation carries the scan held so far
 * and the scan is then retaken from the engine state — the reference builds reset()'s observation before
 * it spins the sensor (crowd_sim_dict.py:166-191), at robot heading 0, against the last human and the
 * world walls. Other envs get the held scan. enable = 0: scans stay zero (config.lidar.enable False).
 * Call after cn_reset / cn_step on the same stream. */
int cn_lidar_obs(cn_engine *eng, void *stream, const uint8_t *reset_mask, int enable, int beams, double max_range,
                 double robot_radius, float *lidar, float *obs);

/* Test hook: the norm-zone predicate of the step kernel, robot 64-gon (GEOS Point.buffer(r)) vs convex quad
 * (crowd_sim.py norm-zone penalty), for n cases on the device: px, py, r [n], qx, qy [n][4],
 * out [n] (1 = intersecting). mode 0: the kernel's function (classification + separating axes), mode 1:
 * the separating-axis test alone. Checked against oracle/cpu_ref.c:disc_quad_intersect in tests/.
 * mode 2: the step kernel's whole norm-zone penalty predicate (both zones built around the robot,
 * crowd_sim.py:918-926): robot at (px, py) of radius r with velocity (qx[i][0], qy[i][0]), float32 heading
 * if qx[i][1] != 0, zone side preference lhs = qy[i][1]. */
int cn_debug_disc_quad(void *stream, int64_t n, int mode, const double *px, const double *py, const double *r,
                       const double *qx, const double *qy, int32_t *out);

/* Test hook (SURVEY Appendix A.4 known answers): agent 0's new velocity of n independent RVO2 simulators
 * of A <= 10 agents each (crowd_nav/policy/orca.py:92-136: addAgent / setAgentPrefVelocity / doStep /
 * getAgentVelocity(0)), through the step kernel's own code path (quad-cooperative neighbour ranking and
 * ORCA lines, linearProgram2, linearProgram3). agents [n][A][5] = (px, py, vx, vy, radius) with agent 0 =
 * self; self [n][3] = (maxSpeed, prefVelocity.x, prefVelocity.y); neighbor_dist, time_horizon, time_step
 * as in PyRVOSimulator. out [n][4] = (vx, vy, index of the line linearProgram2 failed at or the line
 * count when it succeeded, the line count). Checked against oracle/cpu_ref.c:cnref_rvo2_agent0 and hand-derived answers. */
int cn_debug_orca(void *stream, int64_t n, int A, const float *agents, const float *self, float neighbor_dist,
                  float time_horizon, float time_step, float *out);

/* Agent policy plugin (replaces policy_factory[name](config).predict(JointState),
 * crowd_nav/policy/policy_factory.py:1-17; host side crowdnav_dsrnn_amd/policy_factory.py).
 * cn_orca_predict: ORCA.predict (crowd_nav/policy/orca.py:64-139) of n independent simulators of A <= 64
 *   agents, arguments and outputs as cn_debug_orca (the caller keeps the simulator's frozen radii and max
 *   speed, orca.py:85-115). A > 10 runs cn_orca_predict_kd with a fresh simulator's (identity) KdTree order.
 * cn_orca_predict_kd: the same for simulators of A <= 64 agents through RVO2's KdTree (MAX_LEAF_SIZE 10),
 *   whose build re-permutes the simulator's persisted agent order (KdTree::agents_): perm [n][A] uint8 holds
 *   each simulator's order on entry (identity for a simulator created by this predict) and the re-permuted
 *   order on return, so a caller that keeps one simulator across predicts (orca.py:85-90: the simulator
 *   lives until the agent count changes) passes it back next time. perm = NULL: identity, not written.
 *   Caller side: crowd_sim.py:1121-1161 passes N-1 humans (+ the robot when robot.visible), i.e. A = N or N+1.
 * cn_social_force_predict: SOCIAL_FORCE.predict (crowd_nav/policy/social_force.py:11-66) of n agents,
 *   float64: self [n][9] = FullState (px, py, vx, vy, radius, gx, gy, v_pref, theta), others [n][M][5] =
 *   ObservableState (px, py, vx, vy, radius), A / B / KI = config.sf, time_step = config.env.time_step;
 *   out [n][2] = the ActionXY (vx, vy). Device pointers, stream-ordered. */
int cn_orca_predict(void *stream, int64_t n, int A, const float *agents, const float *self, float neighbor_dist,
                    float time_horizon, float time_step, float *out);
int cn_orca_predict_kd(void *stream, int64_t n, int A, const float *agents, const float *self, float neighbor_dist,
                       float time_horizon, float time_step, uint8_t *perm, float *out);
int cn_social_force_predict(void *stream, int64_t n, int M, const double *self, const double *others, double A,
                            double B, double KI, double time_step, double *out);

/* Test hooks of the kd-tree path's resumable spawns (the spawn waves that draw upcoming episodes park a
 * crowded spawn between two humans once a wave has worked `cycles` clock cycles in a launch, and a later
 * launch resumes it; default 600000, 0 = never park; no effect on the quad path, which never parks).
 * cn_debug_spawn_stats: cumulative counts since cn_create [5] = spawns parked before they started, parked
 * mid-way, resumed, completed by a resume (kd-tree path), and auto-resets whose spawn the step kernel drew
 * inline because no pending spawn was ready (every path; synchronises the device). Results do not depend on the budget:
 * tests/test_gpu_parity.py forces parking after every human and compares with the oracle. */
int cn_debug_set_spawn_budget(cn_engine *eng, long long cycles);
int cn_debug_spawn_stats(cn_engine *eng, uint32_t *out);

/* Profiler calibration hook (MI355X_MICROARCH.md § HBM: FETCH_SIZE / WRITE_SIZE are calibrated only for
 * 16-B-per-lane streams): dst[k] = src[k] over n doubles with the step kernel's access shape, one 8-B load
 * and store per lane, in segments of `seg` consecutive doubles per 64-lane wave (seg = 64: a field of the
 * per-human SoA arrays; seg = 6: a per-env field of one workgroup). tools/calib_pmc.py reads the
 * counters of known byte counts through it. */
int cn_debug_copy64(void *stream, int64_t n, int seg, const double *src, double *dst);

/* out[r][h] = sum_n hs[r][n][h] * attn[r][n]; hs [R][N][H], attn [R][N], out [R][H]; H % 4 == 0. */
int cn_attn_pool_fwd(void *stream, int64_t R, int N, int H, const float *hs, const float *attn, float *out);

/* Gradient of cn_attn_pool_fwd: dhs[r][n][h] = dout[r][h] * attn[r][n],
 * dattn[r][n] = sum_h dout[r][h] * hs[r][n][h] (fixed-order reduction). H in {64, 128, 256}. */
int cn_attn_pool_bwd(void *stream, int64_t R, int N, int H, const float *hs, const float *attn, const float *dout,
                     float *dhs, float *dattn);

/* The whole spatial-edge attention of EdgeAttention.forward (srnn_model.py:256-333: spatial_edge_layer,
 * the product with temporal_embed summed over the embedding, * num_edges / sqrt(attention_size), softmax
 * over the N edges, bmm pooling) in one pass over hs, given u = temporal_embed @ Ws [R][H] and
 * c = temporal_embed . bs [R] from the caller (Ws, bs: spatial_edge_layer's weight [A][H] and bias [A]):
 *   attn[r][n] = softmax_n(scale * (hs[r][n] . u[r] + c[r])),  out[r] = sum_n attn[r][n] hs[r][n].
 * hs [R][N][H], out [R][H], attn [R][N]; H in {64, 128, 256}, 1 <= N <= 64; hs, u, out 16-byte aligned. */
int cn_spatial_attn_fwd(void *stream, int64_t R, int N, int H, float scale, const float *hs, const float *u,
                        const float *c, float *out, float *attn);

/* Gradient of cn_spatial_attn_fwd given dout [R][H] and optionally dattn [R][N] (null: none):
 * dhs [R][N][H], du rows of H at stride ldu (-> d temporal_embed = du Ws^T + dc bs^T, dWs = temporal_embed^T du
 * on the caller's side), dc at stride ldc (dc = du + H with ldc = ldu puts [du | dc] in one matrix, so
 * dWs and dbs come from one GEMM). hs, u, dout, dhs, du 16-byte aligned; ldu >= H, ldu % 4 == 0. */
int cn_spatial_attn_bwd(void *stream, int64_t R, int N, int H, float scale, const float *hs, const float *u,
                        const float *attn, const float *dout, const float *dattn, float *dhs, float *du, int64_t ldu,
                        float *dc, int64_t ldc);

/* Weight gradient of a Linear layer over K rows with a tiny side (ops.linear / the fused input layers'
 * backward, replacing torch's dy^T x in the reference's autograd of srnn_model.py:160-161,210-211,466 and
 * distributions.py:74-94): dW[a][j] = sum_k dy'[k][a] x[k][j] and db[a] = sum_k dy'[k][a] with
 * dy' = dy * (relu_out > 0) when relu_out != NULL (the gradient through a ReLU whose output was relu_out).
 * dy, relu_out [K][m], x [K][n] contiguous float32; dW [m][n]; db [m] or NULL; min(m, n) <= 8, max(m, n) <= 256.
 * work: caller-owned device scratch of cn_wgrad_work_elems(K, m, n) floats. Deterministic (fixed order). */
int64_t cn_wgrad_work_elems(int64_t K, int m, int n);
int cn_wgrad(void *stream, int64_t K, int m, int n, const float *dy, const float *relu_out, const float *x,
             float *dW, float *db, float *work);

#ifdef __cplusplus
}
#endif
#endif /* CROWDNAV_H */
