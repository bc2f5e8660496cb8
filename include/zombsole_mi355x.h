/*
 * zombsole_mi355x.h — C ABI of the MI355X-native batched zombsole step engine.
 *
 * The reference (jvstinian/libzombsole) has no FFI: its boundary is the Python
 * class surface ZombsoleGymEnv / MultiagentZombsoleEnv, whose per-tick work is
 * `World.step` plus the env glue.  This header is the seam
 * a maintainer binds from that surface (see INTEGRATION.md for the ctypes
 * stub).  Each entry point names the reference code it replaces:
 *
 *   zs_create      <- ZombsoleGymEnv.__init__ / MultiagentZombsoleEnv.__init__
 *                     (zombsole/gym_env.py:49-83, zombsole/gym/multiagent_env.py:25-78)
 *                     + Game.__init__ (zombsole/game.py:115-140), N envs at once
 *   zs_seed        <- random.seed(s) on the process-global CPython MT19937 the
 *                     reference draws from (/usr/lib/python3.10/random.py:128-168);
 *                     here one independent stream per env
 *   zs_reset       <- env.reset() -> Game.__initialize_world__ + reward reset + obs
 *                     (gym_env.py:148-164, gym/multiagent_env.py:173-184, game.py:151-169)
 *   zs_step        <- env.step(action) (gym_env.py:99-145, gym/multiagent_env.py:111-171):
 *                     set_action, World.step (core.py:72-78), rewards (gym/reward.py),
 *                     respawn (game.py:196-201), observation (gym/observation.py),
 *                     rules (zombsole/rules/{...}.py)
 *   zs_get_state / zs_set_state
 *                  <- the test pokes env.game.world.things, env.game.agents[i].life = x
 *                     (tests/test_game.py:55,105, tests/test_multiagent_env.py:108)
 *   zs_observe     <- env.get_observation() (gym_env.py:93-94)
 *   zs_get_rng / zs_set_rng
 *                  <- random.getstate()/setstate(): the process-global stream the
 *                     reference's World/Game draw from (core.py:2, things.py:2, game.py)
 *   zs_gen_actions <- (bench/parity only) the uniform discrete policy of SURVEY.md §8(d)
 *
 * Conventions: plain C types only; device buffers are raw HIP device pointers,
 * `stream` is a hipStream_t passed as void*.  The engine owns its device
 * state; the caller owns every output buffer.  All calls on one handle are
 * serialized on the stream they are given.  Return value 0 = ok, otherwise a
 * ZS_E* code with a message in zs_last_error() (thread-local).
 */
#ifndef ZOMBSOLE_MI355X_H
#define ZOMBSOLE_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (mapped to Python exceptions by the wrapper) --------- */
#define ZS_OK 0
#define ZS_EINVAL 1    /* -> ValueError                                   */
#define ZS_ENOSPACE 2  /* -> Exception('Not enough space to spawn ...') core.py:62-64 */
#define ZS_EHIP 3      /* -> RuntimeError (HIP failure)                    */
#define ZS_ESTATE 4    /* -> RuntimeError (bad call order / index)         */

/* ---- thing kinds: the observation codes of gym/observation.py:18-26 ---- */
#define ZS_THING_NONE 0
#define ZS_THING_BOX 1
#define ZS_THING_DEADBODY 2
#define ZS_THING_OBJECTIVE 3
#define ZS_THING_WALL 4
#define ZS_THING_ZOMBIE 5
#define ZS_THING_PLAYER 6 /* scripted bot (players/{...}.py)          */
#define ZS_THING_AGENT 7  /* RL agent (players/agent.py)          */

/* ---- weapons: the codes of gym/observation.py:27-34; table weapons.py:18-25 */
#define ZS_WEAPON_NONE 0
#define ZS_WEAPON_CLAWS 1
#define ZS_WEAPON_KNIFE 10
#define ZS_WEAPON_AXE 11
#define ZS_WEAPON_GUN 12
#define ZS_WEAPON_RIFLE 13
#define ZS_WEAPON_SHOTGUN 14
#define ZS_WEAPON_RANDOM 255 /* WeaponFactory 'random' (weapons.py:43-44) */

/* ---- scripted bots (players/{...}.py) -------------------------------------- */
#define ZS_BOT_TERMINATOR 1 /* players/terminator.py */
#define ZS_BOT_SNIPER 2     /* players/sniper.py     */
#define ZS_BOT_TROLL 3      /* players/troll.py      */
#define ZS_BOT_HAMSTER 4    /* players/hamster.py    */
#define ZS_BOT_RANDOMAN 5   /* players/randoman.py   */

/* ---- rules (rules/factory.py:9-19) -------------------------------------- */
#define ZS_RULES_EXTERMINATION 0
#define ZS_RULES_SURVIVAL 1
#define ZS_RULES_EVACUATION 2
#define ZS_RULES_SAFEHOUSE 3

/* ---- agent action kinds (int32 triple kind,dx,dy per agent) ------------- */
#define ZS_ACT_IDLE 0
#define ZS_ACT_MOVE 1
#define ZS_ACT_ATTACK 2
#define ZS_ACT_ATTACK_CLOSEST 3
#define ZS_ACT_HEAL 4
#define ZS_ACT_HEAL_CLOSEST 5
#define ZS_ACT_CONFUSED 6
/* the agent's next_step raises (a debug=True env, core.py:96-99): World.step has advanced t and
 * taken the decisions of the actors before this one in dict order (their RNG draws included), then
 * stops; the env's state is otherwise unchanged and that step reports reward 0, not done, not
 * truncated (the drop-ins re-raise the agent's exception) */
#define ZS_ACT_RAISE 7

/* ---- env surface / observation ------------------------------------------ */
#define ZS_REWARD_SINGLE 0 /* AgentRewards, include_life_in_reward=True (gym/reward.py:19-47) */
#define ZS_REWARD_MULTI 1  /* MultiAgentRewards (gym/reward.py:67-98)                         */
#define ZS_OBS_WORLD 0
#define ZS_OBS_SURROUNDINGS 1
#define ZS_ENC_SIMPLE 0
#define ZS_ENC_CHANNELS 1
#define ZS_DTYPE_I32 0
#define ZS_DTYPE_I64 1
#define ZS_DTYPE_I16 2 /* compact internal form; values fit int16 */

#define ZS_FLAG_AUTORESET 1u /* next-step autoreset: an env that ended is reset by the next zs_step */
#define ZS_FLAG_DEBUG 2u     /* debug=True envs (core.py:96-99, 115-119): action kind ZS_ACT_RAISE
                              * stops World.step; without the flag kinds >= 7 are unknown (idle) */
#define ZS_FLAG_DEATH_LOG 4u /* keep, per env, the things its last step's clean_dead_things removed, in
                              * removal order (zs_death_log; the drop-in views' decoration order and
                              * the final values of a removed zombie whose slot a respawn reuses), and
                              * the actions it executed, in execution order (zs_action_log; the drop-in
                              * views' World.events) */

/* ---- range flags (zs_overflow) -------------------------------------------
 * The reference's obstacle life is an unbounded Python int that carries over resets
 * (game.py:151-155) and keeps falling each time a destroyed Box/Wall is hit again before
 * the first cleanup of an episode (core.py:72-78, 168-184).  The engine holds it in int32. */
#define ZS_OVF_INT16 1u /* an obstacle life went below -32768: ZS_DTYPE_I16 observations saturate it */
#define ZS_OVF_INT32 2u /* an obstacle life reached -2147483647 and saturated there: from then on
                         * that env differs from the reference */

/* ---- map description (parsed by the host; zombsole/game.py:45-97) ------- */
typedef struct zs_map_desc {
    int32_t width, height;
    int32_t n_obstacles;          /* boxes+walls in map-file (dict insertion) order */
    const int32_t* obstacle_xy;   /* [n_obstacles][2]                               */
    const uint8_t* obstacle_kind; /* ZS_THING_BOX / ZS_THING_WALL                   */
    int32_t n_objectives;
    const int32_t* objective_xy;  /* [n][2], map-file order                          */
    int32_t n_player_spawns;
    const int32_t* player_spawn_xy;
    int32_t n_zombie_spawns;      /* 0 => every cell, x-major (core.py:44-47)        */
    const int32_t* zombie_spawn_xy;
} zs_map_desc;

/* ---- launch overrides ----------------------------------------------------------
 * zs_create picks every kernel and layout from the config and the env count.  A non-NULL
 * zs_config.launch forces one of the alternatives it would pick elsewhere, or sizes a grid (parity
 * tests run every alternative; A/B measurements compare them).  Every field: 0 = automatic.
 * Switches: 1 = on, -1 = off.  The block is copied into the handle: no process-wide state, and
 * no environment variable selects a kernel. */
typedef struct zs_launch {
    int32_t fused;           /* reset work inside the step launch (k_step) instead of its own launch  */
    int32_t fobs;            /* observations written by the step launch itself (the default for small
                              * images without a store-stream kernel; -1 off, 1 on)                    */
    int32_t tick_waves;      /* k_tick's register budget: 5 or 6 waves per SIMD                        */
    int32_t lds_budget;      /* -1: largest optional LDS copies instead of the most resident workgroups */
    int32_t rw_need;         /* RNG window words a plain step prefetches (32..512)                    */
    int32_t reset_wgs;       /* reset-work workgroups of a fused step launch                          */
    int32_t reset_stream;    /* -1: an unfused reset launch on the caller's stream, not a side stream  */
    int32_t reset_lists;     /* -1: k_reset reads the spawn lists from HBM instead of LDS              */
    int32_t reset_grid;      /* k_reset workgroups (pending-list mode)                                 */
    int32_t defer_respawn;   /* 1: zombie respawn by k_respawn, -1: by the tick's leader               */
    int32_t respawn_grid;    /* k_respawn workgroups                                                   */
    int32_t obs_pipe;        /* -1: no prefetching store-stream observation kernel (k_obs_pipe family) */
    int32_t obs_lds;         /* the LDS-staged 16-B store kernels (k_obs_patch, k_obs_ring): -1 keeps
                              * k_obs_pipe, 1 takes them at any env count                              */
    int32_t obs_patch;       /* -1: no padded-table encoder kernel k_obs_patch                         */
    int32_t obs_ring;        /* encoder / writer waves through an LDS ring (k_obs_ring, k_obs_pbring);
                              * -1 keeps k_obs_patch / k_obs_pipe / k_obs_gather                       */
    int32_t obs_ring_patch;  /* -1: k_obs_ring with the select-chain encoders instead of the
                              * padded-table ones (its fallback when the tables do not fit)            */
    int32_t obs_gather;      /* -1: no k_obs_gather (large maps then use k_obs)                        */
    int32_t obs_gather_stat; /* -1: k_obs_gather reads static words from HBM instead of LDS tables     */
    int32_t obs_stat;        /* -1: per-cell static words instead of LDS bitmaps                       */
    int32_t obs_win;         /* -1: per-cell entity scan instead of the window map                     */
    int32_t obs_wgs;         /* observation workgroups per CU (store-stream kernels)                   */
    int32_t par_exec;        /* -1: the leader lane executes the shuffled actions serially instead of
                              * the env's lanes in parallel (core.py:103-119)                          */
    int32_t reserved[10];    /* zero (round 6 removed four switches of alternatives measured slower:
                              * the one-launch step k_fstep and its shapes, the early RNG window in
                              * k_tick, the policy inside the side-stream tick)          */
} zs_launch;

typedef struct zs_config {
    int32_t num_envs;
    zs_map_desc map;
    int32_t rules;                /* ZS_RULES_*                                     */
    int32_t num_agents;
    const int32_t* agent_weapons; /* [num_agents] ZS_WEAPON_* or ZS_WEAPON_RANDOM    */
    const int32_t* agent_codes;   /* [num_agents] channels code = 8 + int(agent_id)  */
    int32_t num_bots;
    const int32_t* bot_types;     /* [num_bots] ZS_BOT_* in player_names order       */
    int32_t initial_zombies;
    int32_t minimum_zombies;
    int32_t reward_mode;          /* ZS_REWARD_*                                     */
    int32_t obs_scope;            /* ZS_OBS_*                                        */
    int32_t obs_encoding;         /* ZS_ENC_*                                        */
    int32_t obs_width;            /* surroundings width (odd, > 1)                   */
    int32_t obs_dtype;            /* ZS_DTYPE_*                                      */
    int32_t max_episode_steps;    /* 0 = none; else TimeLimit-style truncation       */
    uint32_t flags;               /* ZS_FLAG_*                                       */
    int32_t lanes_per_env;        /* k_tick lanes per env (1..64, power of 2); 0 = auto */
    const zs_launch* launch;      /* NULL = every launch choice automatic                 */
} zs_config;

typedef struct zs_handle zs_handle;

/* Thread-local message for the last failing call on this thread. */
const char* zs_last_error(void);

/* Validate `cfg`, allocate device state for cfg->num_envs envs on `device`. */
int zs_create(const zs_config* cfg, int device, zs_handle** out);
int zs_destroy(zs_handle* h);

/* Per-env observation shape: out[0] = observations per env (1 for the single
 * surface, num_agents for the multi surface), out[1..3] = C, H, W. */
int zs_obs_shape(const zs_handle* h, int32_t out[4]);

/* CPython random.seed(int) semantics per env, for envs [env0, env0+n).  Host
 * array of n seeds.  Also records the seed as the env's action-stream seed. */
int zs_seed(zs_handle* h, int32_t env0, int32_t n, const uint64_t* seeds_host, void* stream);

/* Reset the envs whose byte in env_mask_dev is nonzero (NULL = all) and write
 * their reset observations into obs_dev (other envs' slices untouched).  A new
 * handle's envs are all pending reset: the first zs_step resets them if zs_reset
 * was not called. */
int zs_reset(zs_handle* h, const uint8_t* env_mask_dev, void* obs_dev, void* stream);

/* Re-encode the observation of the envs whose mask byte is nonzero (NULL = all)
 * from their current state — env.get_observation() (gym_env.py:93-94,
 * gym/multiagent_env.py:87-96), e.g. after a zs_set_state poke. */
int zs_observe(zs_handle* h, const uint8_t* env_mask_dev, void* obs_dev, void* stream);

/* One lock-step tick for every env.
 *   actions_dev      int32 [N][num_agents][3]  (kind, dx, dy)
 *   obs_dev          [N][obs_per_env][C][H][W] of cfg->obs_dtype
 *   rewards_dev      float64 [N][num_agents]   (single surface: [N][1])
 *   done_dev, trunc_dev   uint8 [N]
 *   listed_dev       uint8 [N][num_agents]: agent was in env.agents before the
 *                    step (multi surface: the keys of the returned dicts)
 *   reset_dev        uint8 [N]: 1 when this call reset the env (autoreset)
 * Any output pointer except obs/rewards/done/trunc may be NULL. */
int zs_step(zs_handle* h, const int32_t* actions_dev, void* obs_dev, double* rewards_dev,
            uint8_t* done_dev, uint8_t* trunc_dev, uint8_t* listed_dev, uint8_t* reset_dev,
            void* stream);

/* Bench / parity action stream: actions_dev[e][a] = DISCRETE table entry
 * splitmix64(splitmix64(splitmix64(seed_e) ^ step) ^ a) % n_discrete
 * (libzombsole_amd/actions.py).  n_discrete = 6 or 7. */
int zs_gen_actions(zs_handle* h, uint64_t step, int32_t n_discrete, int32_t* actions_dev,
                   void* stream);

/* The bench loop's step as one replayed hipGraph: zs_gen_actions for step number t, then
 * zs_step (same outputs), where t = step0 on the first call after a (re)capture and advances by
 * one per call on the device.  The launches are captured once per pending-reset-list parity for
 * each set of buffer arguments (the last 4 sets are kept, so double-buffered outputs replay
 * without recapture); results equal zs_gen_actions + zs_step.
 * n_discrete = 0: no policy.  The graph replays zs_step on the caller's actions_dev, which the
 * caller fills on `stream` before each call (a learner's actions, derived from the previous step's
 * observations); results equal zs_step.  This is the graphed form of the reference's per-tick
 * MultiagentZombsoleEnv.step(actions) / ZombsoleGymEnv.step(action) (zombsole/gym/multiagent_env.py:111-171,
 * zombsole/gym_env.py:99-145), one graph launch per step. */
int zs_step_graph(zs_handle* h, uint64_t step0, int32_t n_discrete, int32_t* actions_dev, void* obs_dev,
                  double* rewards_dev, uint8_t* done_dev, uint8_t* trunc_dev, uint8_t* listed_dev,
                  uint8_t* reset_dev, void* stream);
/* n_steps consecutive steps of zs_step_graph in one graph launch (1 <= n_steps <= 64): each step is
 * the same policy launch + zs_step on the same outputs, so the outputs hold the last step's results
 * (a caller that reads every step's outputs takes n_steps = 1).  Saves the per-graph launch gap.
 * With n_discrete = 0 every step of the launch reads the same actions_dev. */
int zs_step_graph_n(zs_handle* h, uint64_t step0, int32_t n_discrete, int32_t n_steps, int32_t* actions_dev,
                    void* obs_dev, double* rewards_dev, uint8_t* done_dev, uint8_t* trunc_dev,
                    uint8_t* listed_dev, uint8_t* reset_dev, void* stream);

/* Host view of one env's state as a flat int32 record (layout below). */
int zs_state_size(const zs_handle* h, int32_t* n_words);
int zs_get_state(zs_handle* h, int32_t env, int32_t* buf_host, void* stream);
int zs_set_state(zs_handle* h, int32_t env, const int32_t* buf_host, void* stream);

/* One env's MT19937 stream in CPython random.getstate() form (625 words: the raw
 * 624-word block being consumed, then the index 0..624 of its next word).  The
 * single-env wrappers move the process-global `random` state through these around
 * every call, so the engine consumes the same global stream the reference draws
 * from (zombsole/core.py:1-2 `import random`; random.py:128-168 getstate/setstate). */
int zs_get_rng(zs_handle* h, int32_t env, uint32_t* state_host, void* stream);
int zs_set_rng(zs_handle* h, int32_t env, const uint32_t* state_host, void* stream);

/* Sticky ZS_OVF_* flags of the handle (everything queued on `stream` included), OR-ed over all
 * envs since zs_create or the last call with clear != 0.  Lossless results need
 * !(flags & ZS_OVF_INT32), and !(flags & ZS_OVF_INT16) for ZS_DTYPE_I16 observations. */
int zs_overflow(zs_handle* h, uint32_t* flags_host, int32_t clear, void* stream);

/* Diagnostics (not part of the reference surface): when enabled, every k_tick
 * (the step kernel), k_obs (the observation kernel) and k_reset (world rebuild)
 * launch is bracketed by HIP events on its stream.  zs_profile_read synchronizes
 * and returns out[0] = total k_tick ms, out[1] = k_tick launches, out[2] = total
 * k_obs ms, out[3] = k_obs launches, out[4] = total k_reset ms, out[5] = k_reset
 * launches, out[6] = total k_respawn ms, out[7] = k_respawn launches (deferred zombie
 * respawns), then clears the record. */
int zs_profile(zs_handle* h, int32_t enable);
int zs_profile_read(zs_handle* h, double out[8]);
/* Diagnostics: the launch configuration the handle chose (lanes per env, LDS images, which
 * observation kernel, fused / side-stream reset work, deferred respawn) as a one-line JSON
 * object, NUL-terminated and truncated to len bytes.  Returns ZS_OK. */
int zs_describe(zs_handle* h, char* buf, int32_t len);
/* Diagnostics: out[0], out[1] = the two pending-reset list counts, out[2] = the deferred-respawn
 * count (after everything queued on stream), out[3] = the list parity the next step drains. */
int zs_debug_lists(zs_handle* h, int32_t out[4], void* stream);
/* The things env's last zs_step removed in World.clean_dead_things (core.py:121-138), in removal order
 * (the dict order at the cleanup): per thing {slot, serial, x, y, life} (its entity record's values at
 * removal), at most cap entries into out_host; *n_out = how many the step removed.  Needs
 * ZS_FLAG_DEATH_LOG; an env reset by that step reports none. */
int zs_death_log(zs_handle* h, int32_t env, int32_t* out_host, int32_t cap, int32_t* n_out, void* stream);
/* The actions env's last zs_step executed, in execution order (World.step's shuffled action list,
 * core.py:76,103-119; replaces reading World.events, core.py:68-70, whose messages the drop-in views
 * derive from it): per action {slot | kind << 8, target} with kind 1 move (target: destination
 * x | y << 16), 2 attack, 3 heal (target: an entity slot, or -1 - obstacle index in map order); at most
 * cap entries into out_host (2 int32 each); *n_out = how many.  Needs ZS_FLAG_DEATH_LOG; an env reset by
 * that step reports none.  A step a debug raise stopped (ZS_ACT_RAISE) reports *n_out = -1 - k and, as its
 * k entries, the actors before the raising one in dict order that decided an action (core.py:80-101: the
 * others were idle). */
int zs_action_log(zs_handle* h, int32_t env, int32_t* out_host, int32_t cap, int32_t* n_out, void* stream);

/* ---- the drop-ins' per-call path ----------------------------------------------------------------
 * ZombsoleGymEnv.step / reset / get_observation and the MultiagentZombsoleEnv equivalents
 * (zombsole/gym_env.py:93-164, zombsole/gym/multiagent_env.py:87-184) run one env per Python call and
 * read everything back on the host.  These calls do that in one host->device copy, the engine's
 * launches, one device->host copy and one synchronisation, on engine-owned device outputs:
 *   zs_host_step(h, actions_host [N][A][3], rng_host, rec_host)  = zs_set_rng + zs_step + read-back
 *   zs_host_reset(h, rng_host, rec_host)                         = zs_set_rng + zs_reset (all envs) + read-back
 *   zs_host_observe(h, rec_host)                                 = zs_observe + read-back
 * rng_host: NULL, or [N][625] words of CPython random.getstate() form moved into the envs' streams
 * before the call (the process-global stream the reference draws from).  rec_host: [N][words] int32
 * records, each with the fixed header below and the sections zs_host_layout gives:
 *   out[0] words per record, out[1] rewards (float64 [R]), out[2] action log (2E words, zs_action_log
 *   form), out[3] death log (5E words, zs_death_log form), out[4] state record (zs_get_state form),
 *   out[5] observation (out[6] bytes, zs_obs_shape of the config's dtype), out[7] R (1 single, A multi).
 * The record always holds the env's stream after the call (rng section), so the caller moves it back into
 * `random` even when zs_host_reset fails with ZS_ENOSPACE. */
#define ZS_HOST_FLAGS 0  /* bit 0 done, bit 1 truncated, bit 2 autoreset by this call                 */
#define ZS_HOST_ERR 1    /* the engine's error word for the call (ZS_ENOSPACE: players could not spawn) */
#define ZS_HOST_ALOG_N 2 /* zs_action_log's n                                                           */
#define ZS_HOST_DLOG_N 3 /* zs_death_log's n                                                            */
#define ZS_HOST_RNG 4    /* 625 words: the env's stream in random.getstate() form                        */
int zs_host_layout(zs_handle* h, int32_t out[8]);
int zs_host_step(zs_handle* h, const int32_t* actions_host, const uint32_t* rng_host, int32_t* rec_host, void* stream);
int zs_host_reset(zs_handle* h, const uint32_t* rng_host, int32_t* rec_host, void* stream);
int zs_host_observe(zs_handle* h, int32_t* rec_host, void* stream);
/* Diagnostic builds compiled with -DZS_STAMPS only (the product .so returns ZS_ESTATE):
 * per-phase k_tick cycle sums / maxima over all workgroup launches since the last call. */
int zs_debug_stamps(zs_handle* h, uint64_t* sum_out, uint64_t* max_out, int32_t n);
/* Diagnostic builds only: out[2w], out[2w + 1] = start / end s_memrealtime (100 MHz) of workgroup w
 * of the last fused step launch (k_step), w < n. */
int zs_debug_timeline(zs_handle* h, uint64_t* out, int32_t n);
/* Diagnostic builds only: out[w * n_phase + k] = cycles of phase k of workgroup w of the step launches
 * since the last zs_debug_stamps / zs_debug_stamps_wg call (the step kernel's slots only), w < n_wgs. */
int zs_debug_stamps_wg(zs_handle* h, uint64_t* out, int32_t n_wgs, int32_t n_phase);

/* Flat state record, int32 words:
 *   [0]  t (World.t)          [1] deaths            [2] zombie_deaths
 *   [3]  episode_steps        [4] n_order (things with ask_for_actions + ... present, dict order)
 *   [5]  needs_reset          [6] n_entities (E)    [7] n_obstacles (O)
 *   [8]  width                [9] height            [10] reward prev zombie_deaths
 *   [11] n_zombies_present    [12] spawn serial counter [13..15] reserved
 *   zs_set_state restores every field except the read-only [6..9], [11]; [5] must equal the
 *   engine's own flag for that env (pending resets are the engine's work lists), else ZS_EINVAL;
 *   an obstacle life below -2147483647 is refused (ZS_EINVAL)
 *   [16 .. 16+8E)  entity records: kind, present, x, y, life, weapon, extra, spawn_serial
 *                  (slots: agents [0,A), bots [A,A+P), zombies [A+P,E))
 *   [.. +E)        order: entity slot ids in dict order (first n_order valid)
 *   [.. +O)        obstacle life      [.. +O) obstacle present (0/1)
 *   [.. +A)        reward tracker previous life per agent
 *   [.. +A)        listed (agent in env.agents) per agent
 *   [.. +ceil(W*H/32)) dead-body bitmap, bit (y*W+x)
 */
#define ZS_STATE_HEADER 16
#define ZS_STATE_ENTITY_WORDS 8

#ifdef __cplusplus
}
#endif
#endif /* ZOMBSOLE_MI355X_H */
