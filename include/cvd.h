/*
 * cvd.h — C-ABI of the MI355X-native Monte-Carlo relative-Viterbi-metric
 * detector (libcvd.so).  Drop-in boundary for the reference's hot path:
 *
 *   reference (So-bonkers/Detecting-Convolutional-Codes-Via-Markovian-Statistics)   this ABI
 *   ───────────────────────────────────────────────────────────────────────────   ─────────────────────
 *   viterbi_markov.py:82-106  branch_output_and_next_state                         cvd_code_tables
 *   viterbi_markov.py:139-159 viterbi_metric_step (Eq. 4-5)                        cvd_metric_step (host), cvd_trace (GPU)
 *   viterbi_markov.py:166-195 enumerate_markov_states_allzero (BFS)                cvd_enumerate (host),
 *                                                                                  cvd_enumerate_device (GPU)
 *   viterbi_markov.py:202-230 + Pd_plotter.py:89-99  T(p) at p = 1/2              cvd_model_* (|Y(i,j)|/2^n, exact)
 *   Pd_plotter.py:123-169     learn_P1_empirical                                   cvd_model_create (host chain),
 *                                                                                  cvd_model_create_device (GPU chain)
 *   viterbi_markov.simulate_markov_sequence (MISSING; called Pd_plotter.py:149,212,219)
 *                                                                                  cvd_generate (+ cvd_trace)
 *   Pd_plotter.py:106-116     log_prob_sequence                                    cvd_detect (per-sequence sums)
 *   Pd_plotter.py:198-233     trial loop, decision, Pd/Pc counting                 cvd_detect (counts) / cvd_mc_run /
 *                                                                                  cvd_mc_fused (generator + table in one kernel)
 *   (none: the reference is single-process)                                        cvd_allreduce_counts / cvd_comm_* (RCCL)
 *   comp_parity.py:90-128     parity_satisfaction_fraction / parity_detector       cvd_parity_detect
 *                             (parity-template baseline)
 *   alpha_exponent.py:83-156  learn_transition_tensor (joint counts)              cvd_count_transitions
 *   alpha_exponent.py:159-188 compute_error_exponent: M(u) for a u grid           cvd_chernoff_build(_dense)
 *   alpha_exponent.py:69-76   spectral_radius (Perron root of M(u) >= 0)           cvd_spectral_radius
 *                             (error-exponent engine)
 *
 * Conventions:
 *   - every function returns 0 on success, a negative CVD_E* code on error;
 *     cvd_last_error() returns a thread-local message; no C++ exception crosses the ABI;
 *   - buffers are caller-owned; pointers named d_* are device pointers (HIP),
 *     `stream` is a hipStream_t (NULL = default stream); launches are async;
 *   - host tables are copied in at cvd_model_create / cvd_model_upload;
 *   - generator taps use the reference layout taps[j][i][d] (output j, input i,
 *     delay d = 0..m; d = 0 multiplies the current input bit), flattened row-major.
 */
#ifndef CVD_H
#define CVD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CVD_ABI_VERSION 11

#define CVD_OK 0
#define CVD_E_INVALID -1      /* bad argument */
#define CVD_E_UNSUPPORTED -2  /* code shape not supported by the requested path */
#define CVD_E_CAPACITY -3     /* enumeration cap hit / table too large */
#define CVD_E_HIP -4          /* HIP runtime error */
#define CVD_E_STATE -5        /* state not in the model's index (reference: KeyError) */

typedef struct cvd_code {
  int32_t k, n, m;         /* inputs, outputs, memory */
  const uint8_t* taps;     /* [n][k][m+1] delay-ordered taps */
} cvd_code;

typedef struct cvd_learn_params {
  double p;                /* BSC crossover of the learning chain */
  int64_t learn_len;       /* < 0: None -> max(5000, 200*S) (Pd_plotter.py:143-146);
                              non-enumerable codes: default_learn_len */
  int64_t learn_burn;      /* Pd_plotter.py:72 default 200 */
  double laplace;          /* Pd_plotter.py:73 default 1.0 */
  uint64_t seed;           /* learning-chain seed (Pd_plotter.py:70 default 12345) */
  int64_t enum_cap;        /* BFS cap; above it the model is sparse (learned states only) */
  int64_t default_learn_len; /* learn length for non-enumerable codes when learn_len < 0 */
  int64_t laplace_states;  /* non-enumerable codes: > 0 = the S of the Laplace denominator S*laplace
                              (Pd_plotter.py:166-167), e.g. a count or certified lower bound from
                              cvd_enumerate_device, >= the visited rows; <= 0 = the visited rows
                              (DESIGN.md D4).  Enumerable codes: <= 0 or the BFS count S. */
} cvd_learn_params;

typedef struct cvd_model_info {
  int32_t kind;            /* 0 = dense (BFS-enumerated, reference-exact), 1 = sparse (learned states) */
  int32_t k, n, m;
  int64_t S;               /* states in the Laplace denominator (BFS count, or learned count) */
  int64_t n_rows;          /* rows held in the device table */
  int64_t learn_len_eff;   /* learning chain length actually used */
  int64_t hash_capacity;   /* explicit-path hash slots (0 if none) */
  int32_t max_probe;       /* longest probe sequence in the hash */
  int32_t device;          /* device holding the tables, -1 if not uploaded */
  double logp1_unseen;     /* log P̂1 of a row never visited (sparse models) */
  int32_t explicit_kernel; /* kernel CVD_PATH_EXPLICIT launches: CVD_KERNEL_* */
  int32_t mc_fused;        /* 1: cvd_mc_run (CVD_PATH_AUTO) runs the fused generator + table kernel
                              (cvd_mc_fused) for this model: an LDS-resident table small enough for
                              256-thread blocks (measured faster there; the 1024-thread variant of the
                              large tables is slower than the two-kernel pipeline) */
  int32_t walk;            /* 1: the specialised m = 6 kernel runs this model's H1 waves in walk mode
                              (learned-row steps from the row records, no ACS; sums unchanged): the
                              model's rows / learn_len < 1/20 (bit-sliced kernel; 1/10 butterfly
                              kernel), i.e. H1 stays in learned rows (CVD_WALK overrides; traces and,
                              unless CVD_WALK=1, counts-only early decision run lockstep) */
  int32_t lds_filter;      /* 1: the specialised kernel keeps this model's whole Bloom filter in LDS
                              (walking models of <= 32,768 rows: 128 KiB in 1,024-thread blocks for the
                              bit-sliced kernel, 64 KiB in 512-thread blocks for the butterfly kernel;
                              CVD_NO_LDSF=1 keeps it in global memory) */
  int32_t walk_compact;    /* 1: the walk reads 8-B two-step records whose log P̂1 values come from a
                              table in LDS beside the filter (built with CVD_WALK_T2C=1 where rows <
                              2^16, <= 4,096 distinct values and room in LDS; same sums, measured
                              neutral, off by default) */
  int64_t multi_variant;   /* nonzero: the specialised kernel variant this model runs in a
                              cvd_detect_multi launch; consecutive models with equal nonzero values
                              share one launch (at most 8), except a model whose own launch would be
                              persistent (persist_seqs below).  0: the model is detected on its own */
  int64_t persist_seqs;    /* > 0: a launch of this model over more sequences than this (the bit-
                              sliced kernel's resident capacity) is persistent -- one block per
                              resident slot, waves taking 64 sequences at a time from a work queue
                              -- and cvd_detect_multi launches it on its own (ABI 10).  0: never */
} cvd_model_info;

#define CVD_KERNEL_NONE 0       /* explicit path unsupported for this shape */
#define CVD_KERNEL_GENERIC 1    /* detect_explicit_kernel<m,k,n>: ACS for every received word */
#define CVD_KERNEL_ORBIT 2      /* detect_k1_kernel<m,n>: k = 1, ACS for the 2^n/2 orbit representatives */
#define CVD_KERNEL_BUTTERFLY 3  /* detect_k1b_kernel<m>: k = 1, n = 2 standard butterflies, one ACS vector */
#define CVD_KERNEL_BUTTERFLY_RTC 4  /* the same, specialised to the decoder code at model upload (JIT, cvd_rtc.cpp) */
#define CVD_KERNEL_BITSLICE_RTC 5   /* m = 6: its bit-sliced form (k1s, cvd_k1s.h: four bit-planes of two words
                                       per lane, the row tables keyed by a canonical digest; same sums) */

typedef struct cvd_model cvd_model;

/* ---- version / errors ---------------------------------------------------- */
int cvd_version(void);
const char* cvd_last_error(void);

/* Stream tag of the (N, p) grid point (the trial streams' Philox counter word 3). */
#define CVD_LEARN_TAG 0xC0DE1EA7u
uint32_t cvd_grid_tag(int64_t N, double p);

/* ---- host-side code algebra (no GPU needed) --------------------------------
 * out_sym[s*2^k + U] = output word (bit j = output j), next_state[s*2^k + U];
 * U = sum_i u_i << i.                                  (viterbi_markov.py:82-106) */
int cvd_code_tables(const cvd_code* code, int32_t* out_sym, int32_t* next_state);

/* One Eq. 4-5 step on the host, D as 2^m bytes.          (viterbi_markov.py:139-159) */
int cvd_metric_step(const cvd_code* dec, const uint8_t* D_prev, int32_t r, uint8_t* D_out);

/* BFS over relative-metric states from D_0 = 0 (viterbi_markov.py:166-195).
 * Writes S; if states_out != NULL it receives [min(S,cap)][2^m] bytes in discovery
 * order; if next_out != NULL, next_out[i*2^n + r] = index of the successor.
 * Returns CVD_E_CAPACITY if more than `cap` states exist. */
int cvd_enumerate(const cvd_code* dec, int64_t cap, int64_t* S_out,
                  uint8_t* states_out, int32_t* next_out);

/* The same BFS on GPU `device` (for codes past the host
 * BFS, (133,171) > 2e8 states): level-synchronous over a hash set in HBM, states in
 * the reference's discovery order (a level's new states ranked by their first
 * (parent, received word) in itertools.product order).  Same outputs as
 * cvd_enumerate (states_out / next_out nullable), plus level_sizes[l] = states
 * first reached after l steps (nullable, max_levels entries; n_levels_out the
 * number of levels).  mem_bytes: device memory budget (<= 0: 90% of free).
 * CVD_E_CAPACITY when S > cap or the budget cannot hold the search: S_out is then
 * a certified lower bound (distinct reachable states found) and the level sizes
 * describe the levels reached.  Synchronous. */
int cvd_enumerate_device(const cvd_code* dec, int32_t device, int64_t cap, int64_t mem_bytes, int64_t* S_out,
                         uint8_t* states_out, int32_t* next_out, int64_t* level_sizes, int32_t max_levels,
                         int32_t* n_levels_out, void* stream);

/* ---- model: decoder trellis + learned P̂1 + T_ref(1/2) ------------------------ */
int cvd_model_create(const cvd_code* dec, const cvd_learn_params* prm, cvd_model** out);
/* The same model with the learning chain (Pd_plotter.py:143-163) run on GPU `device`
 * (parallel in time: speculative blocks verified at their boundaries, first visits
 * by a radix sort of key hashes; see cvd_learn.hip).  Bit-identical to
 * cvd_model_create.  stats_out (nullable) [7]: seconds, mismatched speculative
 * blocks, re-run passes, blocks re-run sequentially, hash/sort attempts,
 * host fallback (1: the GPU chain refused the code shape, the chain length
 * (>= 2^31) or ran out of device memory for its scratch, and the host chain
 * built the model -- identical results), seconds of the sequential tail.
 * Synchronous; `stream` orders the device work (NULL = default stream). */
int cvd_model_create_device(const cvd_code* dec, const cvd_learn_params* prm, int32_t device, void* stream,
                            cvd_model** out, double* stats_out);
int cvd_model_info_get(const cvd_model* model, cvd_model_info* info);
/* Dense models: the S x S P̂1 matrix exactly as Pd_plotter.py:166-167 builds it. */
int cvd_model_dense_P1(const cvd_model* model, double* P_out, int64_t S);
/* Per-row tables (host copies): logP1[row*2^n + r]; keys[row][2^m] metric bytes. */
int cvd_model_rows(const cvd_model* model, double* logp1_out, uint8_t* keys_out, int64_t n_rows);
/* The decoder code of a model (e.g. one loaded from a file): taps_out receives
 * [n][k][m+1] delay-ordered taps (cvd_code layout); len = its size in bytes. */
int cvd_model_taps(const cvd_model* model, uint8_t* taps_out, int64_t len);
int cvd_model_upload(cvd_model* model, int device);
/* The code-specialised detector kernel (CVD_KERNEL_BUTTERFLY_RTC) of an uploaded
 * model: 1 = built, -1 = unavailable (msg_out receives the compiler's reason, the
 * table-driven kernel runs instead with the same results), 0 = not applicable. */
int cvd_model_jit_status(const cvd_model* model, char* msg_out, int64_t msg_len);
void cvd_model_destroy(cvd_model* model);
/* On-disk model cache (the reference memoises P̂1 per learning key with
 * @lru_cache, Pd_plotter.py:123-127; this makes it persistent): save writes the
 * learned rows atomically (tmp + rename); load rebuilds the model (host tables;
 * upload it before use).  Files carry this build's ABI version. */
int cvd_model_save(const cvd_model* model, const char* path);
int cvd_model_load(const char* path, cvd_model** out);

/* ---- device work ---------------------------------------------------------- */
/* Encoder (enc) -> BSC(p) received words for sequences q0..q0+count-1 of an
 * interleaved buffer; sequence q uses
 * seq_id = seq_base + (q - q0) * seq_stride.  Spec of the missing
 * simulate_markov_sequence.  Layout: W = ceil(N / floor(32/n)) words per
 * sequence, step i of a word in bits [n*i, n*i+n); words grouped in 16-byte
 * chunks: word w of sequence q at d_r[((w/4)*pitch + q)*4 + w%4] (16-B aligned);
 * d_r holds ceil(W/4)*4*pitch words. */
int cvd_generate(const cvd_code* enc, uint64_t seed, uint32_t tag, double p, int64_t N,
                 int32_t random_input, int64_t seq_base, int64_t seq_stride,
                 uint32_t* d_r, int64_t pitch, int64_t q0, int64_t count, void* stream);

#define CVD_PATH_AUTO 0
#define CVD_PATH_TABLE 1     /* enumerated state automaton (dense models) */
#define CVD_PATH_EXPLICIT 2  /* explicit 2^m metric vector + hashed P̂1 rows (fastest k=1 kernel that applies) */
#define CVD_PATH_EXPLICIT_GENERIC 3  /* explicit path, ACS for every received word (no orbit reduction) */
#define CVD_PATH_EXPLICIT_ORBIT 4    /* explicit path, k=1 two-representative orbit kernel */
#define CVD_PATH_EXPLICIT_BUTTERFLY 5  /* explicit path, k=1 n=2 butterfly kernel, table-driven (not code-specialised) */
/* OR'ed into `path` (cvd_detect, cvd_mc_run): early decision.  A trial's decision
 * (Pd_plotter.py:215, :222) compares only its final sums; every log P̂1 and log T_ref
 * increment lies in [min, 0], so once the running sums are far enough apart the
 * outcome is certain (with a rigorous IEEE rounding margin) and a wavefront whose
 * lanes have all decided stops.  Counts are identical to the full run; per-trial
 * sums are then not produced (d_sums must be NULL). */
#define CVD_DETECT_EARLY_DECISION 0x100

/* Detector over sequences 0..nseq-1 (pitch = nseq): per sequence the sequential
 * fp64 sums log P̂1(D_0^N) and log T_ref(D_0^N) (Pd_plotter.py:106-116); sequences
 * q < n_h1 are H1 streams (success iff logp1 > logref), the rest H2 streams
 * (success iff logp1 <= logref) (Pd_plotter.py:215-223).  d_counts[0] += H1
 * successes, d_counts[1] += H2 successes (int64, accumulated, not cleared).
 * d_sums (nullable): [nseq][2] doubles.
 * A launch of the bit-sliced kernel past cvd_model_info.persist_seqs is persistent: its
 * waves take their sequences from a work-queue counter the call allocates, zeroes and frees
 * on `stream` (stream-ordered, so launches on any number of streams never share one).
 * Chunked launches (counts only: d_sums NULL, no early decision; the bit-sliced kernel): a
 * batch too small to fill the device twice -- the reference's own call shape, e.g. 10,000
 * trials per p -- has every sequence's N steps cut into C time chunks of L steps, each
 * started on a lane of its own W steps early from D = 0 and kept only where the chunks
 * join (D at a chunk's start equals the previous chunk's D at its end) and the decision is
 * certain under the rounding bounds of both summation orders; every other sequence is rerun
 * on the sequential kernel, so the counts equal the unchunked launch's exactly.  Such a
 * call synchronises `stream` once (the rerun list).  CVD_CHUNK=0 disables it, =1 forces it
 * wherever C >= 2; CVD_CHUNK_WARM (1152 steps) and CVD_CHUNK_UNITS set W and the target lane
 * count. */
int cvd_detect(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq,
               int64_t n_h1, double* d_sums, int64_t* d_counts, int32_t path, void* stream);

/* nm cvd_detect calls in as few launches as possible (a p sweep: one model per p, one
 * stream buffer each; Pd_plotter.py:199-233).  Model i reads d_r[i] (nseq[i] sequences,
 * the first n_h1[i] of them H1) and accumulates d_counts[i][2] (and d_sums[i] when d_sums
 * and d_sums[i] are non-NULL), all with the same N.  Consecutive models that share the
 * code-specialised kernel variant (CVD_KERNEL_BUTTERFLY_RTC: same decoder, block size
 * and filter placement) run in ONE launch, up to 8 per launch, block ranges in model
 * order, so the step pays one last-round tail instead of one per model; others run as
 * cvd_detect.  Results equal the separate calls exactly.  path: CVD_PATH_AUTO or
 * CVD_PATH_EXPLICIT (merged), any other path launches one model at a time; OR
 * CVD_DETECT_EARLY_DECISION as in cvd_detect.  CVD_NO_MULTI=1 disables merging. */
int cvd_detect_multi(const cvd_model* const* models, int32_t nm, const uint32_t* const* d_r, int64_t N,
                     const int64_t* nseq, const int64_t* n_h1, double* const* d_sums, int64_t* const* d_counts,
                     int32_t path, void* stream);

/* Metric trace on the explicit path: d_D[(t*nseq + q)*2^m + s] = D_t(s), t = 0..N. */
int cvd_trace(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq,
              uint8_t* d_D, void* stream);

/* One (N, p) grid point over global trials [trial_begin, trial_end): generates
 * H1 (enc1) and H2 (enc2) streams in batches of `batch` trials into the caller's
 * workspace d_work (cvd_mc_workspace_bytes) and accumulates d_counts[2]. */
int64_t cvd_mc_workspace_bytes(const cvd_code* enc1, int64_t N, int64_t batch);
int cvd_mc_run(const cvd_model* model, const cvd_code* enc1, const cvd_code* enc2,
               double p, int64_t N, uint64_t seed, int64_t trial_begin, int64_t trial_end,
               int64_t batch, void* d_work, int64_t* d_counts, int32_t path, void* stream);

/* cvd_mc_run: d_work may be NULL when the call runs the fused kernel below (CVD_PATH_AUTO
 * and cvd_model_info.mc_fused); otherwise it returns CVD_E_INVALID without it.  The fused
 * path launches at most 2^28 trials per kernel (HIP grid limit), in slices. */

/* The whole (N, p) grid of Pd_plotter.py:196-233 in one call: N outer,
 * p inner, the global trials [trial_begin, trial_end) at every point (the reference's
 * num_iter per point; a shard of them under trial sharding), with models[i] the model
 * learned at p[i] (learn_P1_empirical is per p, Pd_plotter.py:123-169).  Point
 * (N[j], p[i]) accumulates into d_counts[(j*np + i)*2 + {0: H1, 1: H2}] -- the
 * [nN][np][2] count tensor cvd_allreduce_counts reduces -- exactly the counts np * nN
 * cvd_mc_run calls give.  The p row of one N runs batch by batch: every point's streams
 * are generated into its own workspace slot, then one cvd_detect_multi detects the row
 * (the models sharing the specialised kernel variant in one launch, so a row of small
 * batches -- the reference's num_iter = 10,000 per point -- pays one last-round tail,
 * not one per p); points whose model runs the fused kernel (CVD_PATH_AUTO, mc_fused)
 * run it without a slot.  d_work: cvd_mc_grid_workspace_bytes (one slot of the largest
 * N's batch per non-fused point; 0 = NULL allowed when every point runs fused). */
int64_t cvd_mc_grid_workspace_bytes(const cvd_model* const* models, int32_t np, const cvd_code* enc1,
                                    const int64_t* N, int32_t nN, int64_t batch, int32_t path);
int cvd_mc_run_grid(const cvd_model* const* models, const cvd_code* enc1, const cvd_code* enc2,
                    const double* p, int32_t np, const int64_t* N, int32_t nN, uint64_t seed,
                    int64_t trial_begin, int64_t trial_end, int64_t batch, void* d_work,
                    int64_t* d_counts, int32_t path, void* stream);

/* Kernel error flags of a model's launches since the last call (synchronises its
 * device): bit 0 = a walk-mode wave (k1b_walk) left its scheduler loop by the guard
 * bound with lanes unfinished, so that launch's counts and sums are void.  Returns
 * CVD_E_STATE when any flag is set (then cleared), CVD_OK otherwise.  cvd_detect,
 * cvd_detect_multi, cvd_mc_run and cvd_mc_run_grid do not synchronise, so they cannot
 * report it: a caller checks it once after its launches (the Python host does after
 * run_trials with sums, run_grid, detect_multi's callers, run_experiment and the bench). */
int cvd_model_device_error(cvd_model* model, int32_t* flags_out);

/* The chunked launches of this process's last cvd_detect / cvd_detect_multi call (cvd_mc_run
 * and cvd_mc_run_grid make such calls per batch): out[0] chunked launch groups (0: none),
 * out[1] chunks per sequence C, out[2] steps per chunk L, out[3] sequences the decisions
 * left to the sequential rerun.  Diagnostic (tests, bench); not thread-safe. */
int cvd_chunk_last(int64_t* out4);

/* Compile the code-specialised detector's default variants for decoder `dec` and GPU
 * architecture `arch` (e.g. "gfx950") into `dir` without a device: the prebuilt cache that
 * model upload reads before compiling (its default: <directory of libcvd.so>/jit;
 * CVD_JIT_PREBUILT=off skips it).  Only the bit-sliced codes (m = 6, k = 1, n = 2 standard
 * butterflies) have variants to build; *n_built = how many were built or found. */
int cvd_jit_prebuild(const cvd_code* dec, const char* arch, const char* dir, int32_t* n_built);

/* The same grid point in ONE kernel per launch, without streams in HBM: every lane
 * generates its own sequence's received words (cvd_generate's encoder and noise, bit
 * for bit) and runs the LDS-resident table automaton on them (dense models with
 * S < 4096 whose tables fit a CU's LDS; (k, n) in {(1,2), (1,3), (2,3)}; otherwise
 * CVD_E_UNSUPPORTED).  Trial t of [trial_begin, trial_end) is sequences 2t (H1, enc1)
 * and 2t + 1 (H2, enc2) as in cvd_mc_run, which uses this path for CVD_PATH_AUTO
 * when it applies.  d_sums (nullable): [trial_end - trial_begin][4] doubles (log P̂1,
 * log T_ref of H1, then of H2).  flags: CVD_DETECT_EARLY_DECISION (counts only). */
int cvd_mc_fused(const cvd_model* model, const cvd_code* enc1, const cvd_code* enc2, double p, int64_t N,
                 uint64_t seed, int64_t trial_begin, int64_t trial_end, double* d_sums, int64_t* d_counts,
                 int32_t flags, void* stream);

/* ---- multi-GPU: the one collective (none in the reference,
 * Pd_plotter.py:176-235 is single-process) --------------------------------
 * Sum-reduce the int64 success counts of a trial-sharded run over RCCL (xGMI).
 * Shard the global trial range [0, num_iter) of every (N, p) grid point over the
 * GPUs, run cvd_mc_run per shard into a per-device count buffer, reduce: every
 * buffer then holds the single-process counts (streams are keyed by the global
 * trial id).  Enqueued on the given streams (async; the caller synchronises).
 *
 * One process, ndev devices: d_counts[i] on devices[i], ordered after streams[i]
 * (streams NULL or streams[i] NULL = that device's default stream).  The
 * communicators are created on first use of a device list and cached. */
int cvd_allreduce_counts(int64_t* const* d_counts, int64_t len, int32_t ndev, const int32_t* devices,
                         void* const* streams);
/* One process per GPU: rank 0 calls cvd_comm_unique_id and hands the 128 bytes to
 * every rank (any channel); each rank calls cvd_comm_init with its device. */
#define CVD_COMM_ID_BYTES 128
typedef struct cvd_comm cvd_comm;
int cvd_comm_unique_id(uint8_t* id_out /* [CVD_COMM_ID_BYTES] */);
int cvd_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, cvd_comm** out);
int cvd_comm_allreduce_counts(cvd_comm* comm, int64_t* d_counts, int64_t len, void* stream);
void cvd_comm_destroy(cvd_comm* comm);

/* ---- parity-template baseline (comp_parity.py, parity_eqn_check.py) --------
 * Per sequence q of a received-word buffer (pitch = nseq, layout as above):
 *   sat = #{t in [max_s, N) : XOR_{(j,s) in terms} y_j[t - s] == 0}
 * with y_j[t] = bit j of step t (comp_parity.py:90-117: anchors from the
 * template's largest delay max_s), P̂ = sat / (N - max_s), 0.0 without anchors.
 * Sequences q < n_h1 succeed iff P̂ >= gamma (decide H1), the rest iff P̂ < gamma
 * (comp_parity.py:120-128); d_counts[2] accumulated as in cvd_detect.
 * terms: [n_terms][2] (output j, delay s), 1 <= n <= 3, 1 <= n_terms <= 64,
 * 0 <= s <= 64 - floor(32/n).  d_sat (nullable): [nseq] int32 satisfied counts. */
int cvd_parity_detect(const uint32_t* d_r, int32_t n, int64_t N, int64_t nseq, int64_t n_h1,
                      const int32_t* terms, int32_t n_terms, double gamma, int32_t* d_sat,
                      int64_t* d_counts, void* stream);

/* ---- error-exponent engine (alpha_exponent.py, Eq. 7) ---------------------
 * Joint counts of (metric state i, received word r) along received streams
 * (pitch = nseq) for steps t >= burn_in, on a dense (enumerated) model with
 * S < 4096: d_cnt[i*2^n + r] += count (uint64, accumulated, not cleared).
 * The chain's next state is the model's automaton (alpha_exponent.py:136-149). */
int cvd_count_transitions(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq,
                          int64_t burn_in, uint64_t* d_cnt, void* stream);
/* M(u) = sum_r P1(i->j,r)^u P2(i->j,r)^(1-u) for u = d_u[0..U) from joint counts
 * cnt1/cnt2 [K*R] (f64) of tensors P = (C + laplace) / rowsum over (j, r)
 * (alpha_exponent.py:152-154), C[i,j,r] = cnt[i,r] iff j = next(i,r): written as
 * d_a[U*K] (rank-one part, M += a 1^T) and d_vals[U*K*R] (entry (i, next(i,r))). */
int cvd_chernoff_build(int32_t K, int32_t R, const double* d_cnt1, const double* d_cnt2, double laplace,
                       const double* d_u, int32_t U, double* d_a, double* d_vals, void* stream);
/* Dense M(u)[i][j] (d_vals[U*K*K]) from arbitrary P1, P2 [K*K*R] (alpha_exponent.py:170-180). */
int cvd_chernoff_build_dense(int32_t K, int32_t R, const double* d_P1, const double* d_P2,
                             const double* d_u, int32_t U, double* d_vals, void* stream);
/* Perron root of each of U nonnegative K x K matrices M = a 1^T + ELL(vals, cols)
 * (E entries per row; d_cols NULL: dense rows, E = K; d_a NULL: no rank-one part)
 * by power iteration with Collatz-Wielandt bounds: d_rho[3u..3u+2] = (estimate,
 * lower, upper bound) once (upper - lower) <= tol * upper (irreducible M), else
 * once the power-iteration norm ratio is stable to tol/100 (the estimate), or
 * after max_iter iterations (d_iters[u]).  K <= 10000: vectors in LDS, one workgroup per u;
 * larger K (structured form only, d_cols non-NULL): vectors in HBM, one launch per phase. */
int cvd_spectral_radius(int32_t K, int32_t E, const double* d_a, const double* d_vals,
                        const int32_t* d_cols, int32_t U, double tol, int32_t max_iter, double* d_rho,
                        int32_t* d_iters, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CVD_H */
