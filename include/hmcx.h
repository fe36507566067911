/* hmcx.h — C ABI of the MI355X-native SG-HMC engine (libhmcx.so).
 *
 * The reference (sherna90/dropout_hamiltonian_montecarlo) has no FFI: its boundary is a
 * duck-typed Python protocol.  This header is the boundary the Python host
 * layer (dropout_hamiltonian_montecarlo_amd/hamiltonian/...) binds through ctypes; each
 * entry point names the reference interface it replaces.
 *
 * Conventions
 *  - All array pointers are DEVICE pointers (caller-owned, e.g. torch tensors), row-major
 *    and contiguous, unless the comment says "host".
 *  - C independent chains are stored chain-interleaved so the two gradient GEMMs see one
 *    [rows x C*K] matrix: weights W[D][C][K], bias b[C][K]  (C = 1 is exactly the
 *    reference's {'weights': [D,K], 'bias': [K]} layout).
 *  - dtype: HMCX_F64 (the reference's float64) or HMCX_F32.
 *  - Return 0 on success or a negative hmcx_status; hmcx_last_error() has the message.
 *    No C++ exception crosses the ABI.  A context is bound to one device, owns its
 *    workspace and (unless hmcx_set_stream is used) its HIP stream; it is not thread-safe.
 *  - Every call is asynchronous on the context stream; results are ready after
 *    hmcx_synchronize() (or any stream-ordered consumer).
 */
#ifndef HMCX_H
#define HMCX_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hmcx_ctx hmcx_ctx;

enum hmcx_dtype { HMCX_F32 = 0, HMCX_F64 = 1 };
enum hmcx_noise { HMCX_NOISE_BUFFER = 0, HMCX_NOISE_PHILOX = 1 };
enum hmcx_status {
  HMCX_OK = 0,
  HMCX_EINVAL = -1,       /* bad argument / shape */
  HMCX_EHIP = -2,         /* HIP runtime error */
  HMCX_ENOMEM = -3,       /* device allocation failed */
  HMCX_EUNSUPPORTED = -4  /* shape/dtype combination not built */
};

/* ------------------------------------------------------------------ context */
int hmcx_version(void);
int hmcx_create(int device, hmcx_ctx** out);
int hmcx_destroy(hmcx_ctx* ctx);
const char* hmcx_last_error(const hmcx_ctx* ctx);
/* Run on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = the legacy
 * default stream.  A new context runs on its own non-blocking stream until this is called. */
int hmcx_set_stream(hmcx_ctx* ctx, void* hip_stream);
int hmcx_synchronize(hmcx_ctx* ctx);
/* Capture each hmcx_*_run call into a hipGraph and replay it (1) or launch eagerly (0). */
int hmcx_set_graph_mode(hmcx_ctx* ctx, int enabled);
/* SGHMC implementation: 0 = auto (persistent single-launch kernel when C == 1 and the shape
 * fits, else kernel-per-phase), 1 = kernel-per-phase, 2 = persistent only (error otherwise). */
int hmcx_set_sghmc_path(hmcx_ctx* ctx, int path);
/* Device timing of sampler runs: when enabled, HIP events on the launch stream bracket the
 * kernels of every hmcx_sghmc_run / hmcx_sgld_run call (for the persistent SGHMC path: exactly
 * its one kernel launch).  Enabling (or disabling) resets the totals; hmcx_get_timing waits
 * for the last bracketed run and returns the summed kernel time and the number of runs. */
int hmcx_set_timing(hmcx_ctx* ctx, int enabled);
int hmcx_get_timing(hmcx_ctx* ctx, double* kernel_ms, long long* launches);

/* Philox4x32-10 uniforms in [0,1), bit-identical to the device generator (host function). */
void hmcx_philox_uniforms(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                          uint32_t n, double* out /* host [n] */);
/* Philox standard normals for slot/element range (host function; used by tests): the float32
 * Box–Muller stream of the f32 chains. */
void hmcx_philox_normals(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                         uint32_t e0, uint32_t n, double* out /* host [n] */);
/* The float64 stream of the f64 chains (53-bit uniforms, double Box–Muller; host function).
 * Replaces the f64 draws of cpu/sghmc.py:21,31 and cpu/sgld.py:45 in noise='philox' mode. */
void hmcx_philox_normals_f64(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                             uint32_t e0, uint32_t n, double* out /* host [n] */);

/* ------------------------------------------------------------------ softmax model
 * Replaces hamiltonian/models/cpu/softmax.py:45-61 (grad) and gpu/softmax.py:53-69.
 * X [B][D], Y [B][K] one-hot (dtype), W [D][C*K], b [C*K]  ->  gW [D][C*K], gb [C*K]
 * grad = -(Xᵀ(Y - softmax(clip(XW+b))) - alpha*theta)                                  */
int hmcx_softmax_grad(hmcx_ctx* ctx, int dtype, const void* X, const void* Y, int B, int D, int K,
                      int C, const void* W, const void* b, double alpha, void* gW, void* gb);

/* Replaces softmax.py:63-72 (log_likelihood): ll[c] = Σ_rows Σ_k y·(z − logsumexp z), z = clip(XW+b).
 * ll: device double[C]. */
int hmcx_softmax_loglik(hmcx_ctx* ctx, int dtype, const void* X, const void* Y, int B, int D, int K,
                        int C, const void* W, const void* b, double* ll);

/* Replaces softmax.py:38-43,82-89 (net / predict(prob=True)): prob [B][C*K]. */
int hmcx_softmax_predict(hmcx_ctx* ctx, int dtype, const void* X, int B, int D, int K, int C,
                         const void* W, const void* b, void* prob);

/* ------------------------------------------------------------------ logistic model
 * Replaces hamiltonian/models/cpu/logistic.py:24-72 (K = 1; the GPU file models/gpu/logistic.py is
 * its CuPy twin).  X [B][D], y [B] (dtype, 0/1), W [D][C], b [C] (C independent parameter sets, C = 1
 * is the reference's {'weights': [D,1], 'bias': [1]}).
 * net = sigmoid(clip(XW + b)) = 1/(1 + exp(−z)) (:43-55);  grad = −(Xᵀ(y − net) − alpha·θ) (:24-41). */
int hmcx_logistic_grad(hmcx_ctx* ctx, int dtype, const void* X, const void* y, int B, int D, int C,
                       const void* W, const void* b, double alpha, void* gW, void* gb);
/* ll[c] = Σ_rows y·log(net) + (1 − y)·log(1 − net)  (:64-72), device double[C]. */
int hmcx_logistic_loglik(hmcx_ctx* ctx, int dtype, const void* X, const void* y, int B, int D, int C,
                         const void* W, const void* b, double* ll);
/* prob [B][C] = net (predict(prob=True) of :75-87, before batching). */
int hmcx_logistic_predict(hmcx_ctx* ctx, int dtype, const void* X, int B, int D, int C, const void* W,
                          const void* b, void* prob);
/* out[0] = Σ x² (float64 accumulation, fixed order): the θ-dependent part of logistic.log_prior
 * (:15-21).  x device [n] (dtype), out device double[1]. */
int hmcx_sumsq(hmcx_ctx* ctx, int dtype, const void* x, int64_t n, double* out);

/* ------------------------------------------------------------------ momentum SGD (sgd.fit)
 * Replaces hamiltonian/inference/cpu/sgd.py:25-45 (fit) and :47-70 (fit_dropout) for the softmax
 * and logistic models: per minibatch s (rows row0[s] .. +B of X / Y)
 *   g = model.grad(θ, X_s, Y_s);  m = gamma·m − step_size·g;  θ += m      (sgd.py:38-41)
 * with X_s replaced by X_s ⊙ Z (Z ∈ {0,1}^{B×D}) when dropout is set (sgd.py:61-63).  Z comes from
 * keep (device uint8, B·D per step from keep_off[s]; BUFFER: the host's np.random.binomial draws)
 * or from Philox (PHILOX: Z = u < keep_p, u = Philox(seed, 0, step_base + s, 0xFFFFFFFC, element)). */
enum hmcx_model { HMCX_MODEL_SOFTMAX = 0, HMCX_MODEL_LOGISTIC = 1 };
typedef struct hmcx_sgd_args {
  int dtype;
  int model;               /* hmcx_model                                                  */
  int B, D, K, n_steps;    /* K = 1 for the logistic model                                */
  double alpha;            /* prior precision (hyper['alpha'])                            */
  double step_size;        /* sgd.py:14                                                   */
  double gamma;            /* momentum decay, sgd.py:25                                   */
  const void* X;           /* device [N][D]                                               */
  const void* Y;           /* device [N][K] (softmax one-hot) or [N] (logistic)           */
  const int64_t* row0;     /* host [n_steps]                                              */
  int dropout;             /* 0: fit, 1: fit_dropout                                      */
  double keep_p;           /* fit_dropout's p (PHILOX mode)                               */
  int mask_mode;           /* HMCX_NOISE_BUFFER or HMCX_NOISE_PHILOX                      */
  const uint8_t* keep;     /* device, BUFFER                                              */
  const int64_t* keep_off; /* host [n_steps], BUFFER                                      */
  uint64_t seed;           /* PHILOX                                                      */
  uint32_t step_base;      /* PHILOX                                                      */
  void* W; void* b;        /* device state [D][K], [K], updated in place                  */
  void* mW; void* mb;      /* device momentum (zero at fit start, sgd.py:35)              */
} hmcx_sgd_args;
int hmcx_sgd_run(hmcx_ctx* ctx, const hmcx_sgd_args* a);

/* ------------------------------------------------------------------ samplers
 * One call enqueues n_steps consecutive sampler steps for C chains that share each
 * minibatch; the minibatch of step s is rows [row0[s], row0[s]+B) of X / Y.
 * noise_mode BUFFER: `noise` (device double) holds standard normals; the block of
 * (step s, chain c) starts at noise_off[s*C+c] and is laid out exactly in the
 * reference's draw order, P = D*K + K values per draw: SGHMC = momentum then one
 * draw per leapfrog iteration (weights then bias each); SGLD = one draw per step.
 * noise_mode PHILOX: normals come from Philox(seed, chain0+c, step_base+s, slot, elem). */
typedef struct hmcx_sampler_args {
  int dtype;
  int B, D, K, C;          /* minibatch rows, features, classes, chains in this call   */
  int n_steps;
  double alpha;            /* Gaussian prior precision (hyper['alpha'])               */
  double log_prior;        /* constant log_prior (cpu softmax.py:22-30), host-computed */
  const void* X;           /* device [N][D] (dtype)                                    */
  const void* Y;           /* device [N][K] (dtype, one-hot)                           */
  const int64_t* row0;     /* host [n_steps]                                           */
  const double* eps;       /* host [n_steps]  step size used by step s                */
  const int32_t* n_iter;   /* host [n_steps*C] SGHMC leapfrog iterations max(0, L-1)   */
  const double* u_accept;  /* host [n_steps*C] accept uniforms (SGHMC); both NULL in    */
                           /* PHILOX mode: drawn by the call (path_length, out_L)       */
  const uint8_t* want_ll;  /* host [n_steps] or NULL: SGLD computes ll(q_new) after s  */
  int noise_mode;
  const double* noise;     /* device, BUFFER mode                                      */
  const int64_t* noise_off;/* host [n_steps*C], BUFFER mode                            */
  uint64_t seed;           /* PHILOX mode                                              */
  uint32_t chain0;         /* PHILOX: global id of chain 0 of this call               */
  uint32_t step_base;      /* PHILOX: global step id of step 0 of this call           */
  void* W;                 /* device [D][C*K] state, updated in place                  */
  void* b;                 /* device [C*K]                                              */
  double* out_A;           /* device [n_steps*C] accept probability (SGHMC)            */
  int32_t* out_accepted;   /* device [n_steps*C]                                       */
  double* out_ll;          /* device [n_steps*C] log_likelihood(q_after, batch)        */
  double* out_E;           /* device [n_steps*C*2] (E_current, E_new) or NULL          */
  void* pW;                /* SGLD only, or NULL: device [D][C*K] momentum carried     */
  void* pb;                /*   across steps; selects the CuPy file's update (A2g)     */
  void* out_trace;         /* device [n_steps][C][D*K+K] (dtype) or NULL: the state     */
                           /* after every step (weights row-major, then bias) — the rows */
                           /* of the HDF5 backend (sghmc_multicore.py:49-51)            */
  int32_t* out_abort;      /* device [1] or NULL (SGHMC): 0, or 1 when a persistent launch */
                           /* timed out in a hand-off (or followed one that did) and left */
                           /* W/b untouched — see hmcx_clear_abort.  NULL: the check is    */
                           /* deferred to the next call / hmcx_synchronize instead.       */
                           /* SGLD (wide path): 1 when a fused team round timed out; W/b  */
                           /* are then invalid (hmcx_set_sgld_fuse).  NULL: the call re-runs */
                           /* itself and waits for its stream.                            */
  double path_length;      /* SGHMC, PHILOX mode with n_iter == u_accept == NULL: the call */
  double* out_L;           /* draws its own schedule (hmcx_philox_schedule, this path     */
                           /* length); out_L (host [n_steps*C] or NULL) receives the L's  */
  void* out_mom;           /* SGHMC, C < 16, or NULL: device [C][D*K+K] (dtype), the       */
                           /* momentum the call's LAST step returns (sghmc.py:36-39): the */
                           /* final p_new if accepted, else the drawn p                   */
  void* out_host;          /* SGHMC or NULL: pinned host block that receives the call's     */
                           /* outputs once the launch has finished: [n_steps*C f64 A]      */
                           /* [.. f64 ll][2*n_steps*C f64 E][n_steps*C i32 accepted][i32   */
                           /* abort].  out_A/out_ll/out_E/out_accepted must then be that    */
                           /* layout in one device block; the call copies it behind its     */
                           /* kernels (one copy when out_abort is the i32 right after that  */
                           /* block, else two) and records an event: hmcx_host_wait.        */
} hmcx_sampler_args;

/* Replaces hamiltonian/inference/{cpu,gpu}/sghmc.py:19-39 (step, with the A1 completion:
 * momentum ~ N(0,1), MH accept min(1, exp(E_cur - E_new)) from cpu/hmc.py:67-87). */
int hmcx_sghmc_run(hmcx_ctx* ctx, const hmcx_sampler_args* a);

/* Blocks until the outputs of the latest hmcx_sghmc_run call that named this out_host block have
 * landed in it (an event recorded behind that call's copies; no stream-wide synchronisation, so
 * calls enqueued after it keep running).  A block no call has named returns at once. */
int hmcx_host_wait(hmcx_ctx* ctx, const void* out_host);

/* Persistent-kernel hand-off timeouts (single-chain SGHMC).  A launch whose workgroups time out
 * waiting for each other (they were not co-resident, or not placed on the XCDs the kernel assumes)
 * writes nothing to W/b and raises the context's abort word; every later persistent launch sees the
 * raised word and returns at once, also without touching W/b.  The caller re-runs those calls (in
 * order, e.g. on the kernel-per-phase path: hmcx_set_sghmc_path(ctx, 1)) after hmcx_clear_abort,
 * which lowers the word (stream-ordered) and drops the deferred checks still pending. */
int hmcx_clear_abort(hmcx_ctx* ctx);

/* Fallback bookkeeping.  Every path that re-runs work after a timed-out cross-workgroup exchange
 * is counted per context, so a test suite, smoke check or benchmark can require that none happened
 * (a re-run gives the right result, which is exactly why it must not go unnoticed):
 *   HMCX_RECOVERY_PERSISTENT  persistent SGHMC calls re-run after a timed-out launch (hmcx_clear_abort
 *                             itself counts nothing; the host code that re-runs records each call)
 *   HMCX_RECOVERY_MLP_FUSED   hmcx_mlp_sghmc_run calls re-run unfused after their out_abort verdict
 *                             (the host code that re-runs records it: hmcx_note_recovery)
 *   HMCX_RECOVERY_WIDE_FUSED  hmcx_sgld_run calls whose fused forward + softmax timed out and that
 *                             re-ran on the three-launch path inside the call
 * counts: host int64_t[HMCX_RECOVERY_KINDS], totals since hmcx_create. */
enum hmcx_recovery {
  HMCX_RECOVERY_PERSISTENT = 0,
  HMCX_RECOVERY_MLP_FUSED = 1,
  HMCX_RECOVERY_WIDE_FUSED = 2,
  HMCX_RECOVERY_KINDS = 3
};
int hmcx_get_recoveries(const hmcx_ctx* ctx, int64_t* counts);
int hmcx_note_recovery(hmcx_ctx* ctx, int kind);

/* Host-side Philox schedule of noise='philox' SGHMC steps (sghmc.py:25 path length, :36 accept
 * uniform), bit-identical to the device generator: for step s < n_steps and chain c < C
 *   L[s*C+c] = ceil(2·u_path·path_length / eps[s]),  n_iter = max(0, L − 1),  u = u_accept
 * with u_path / u_accept = Philox(seed, chain0 + c, step_base + s, SLOT_PATH / SLOT_ACCEPT, 0).
 * All arrays host.  Returns HMCX_EINVAL for a non-finite or oversized path length. */
int hmcx_philox_schedule(uint64_t seed, uint32_t chain0, int C, uint32_t step_base, int n_steps,
                         double path_length, const double* eps, double* L, int32_t* n_iter, double* u);

/* Replaces hamiltonian/inference/cpu/sgld.py:31-46 (step): p = N(0,(2ε)²) − ½ε∇U; q += p.
 * With pW/pb set: hamiltonian/inference/gpu/sgld.py:11-20, p = ν⊙p_prev − ½ε∇U with
 * ν ~ N(0,(2ε)²), q += p, p written back to pW/pb. */
int hmcx_sgld_run(hmcx_ctx* ctx, const hmcx_sampler_args* a);

/* ------------------------------------------------------------------ full-batch HMC, MVN model
 * Replaces cpu/hmc.py:39-64 with models/cpu/mvn_gaussian.py (config 1).
 * x [C][dim] state; mu [dim]; prec [dim][dim] = inv(cov); nlp_const = dim·log2π + log det cov,
 * nlp(x) = 0.5·(nlp_const + (x−μ)ᵀ·prec·(x−μ))  (mvn_gaussian.py:27-30 op order).
 * momentum/accept randomness as in hmcx_sampler_args (BUFFER: noise_off per step/chain, dim
 * normals per step).  out_nlp = nlp(q after step). */
typedef struct hmcx_hmc_mvn_args {
  int dim, C, n_steps;
  const double* mu;        /* device [dim] */
  const double* prec;      /* device [dim][dim] */
  double nlp_const;
  const double* eps;       /* host [n_steps] */
  const int32_t* n_iter;   /* host [n_steps*C] */
  const double* u_accept;  /* host [n_steps*C] */
  int noise_mode;
  const double* noise;
  const int64_t* noise_off;
  uint64_t seed;
  uint32_t chain0, step_base;
  double* x;               /* device [C][dim] */
  double* out_A;
  int32_t* out_accepted;
  double* out_nlp;
  double* out_trace;       /* device [n_steps][C][dim] or NULL */
} hmcx_hmc_mvn_args;
int hmcx_hmc_mvn_run(hmcx_ctx* ctx, const hmcx_hmc_mvn_args* a);
/* Per-call MVN surface, mvn_gaussian.py:14-31: for C points x [C][dim], g = (x − μ)·prec (grad) and
 * nlp = 0.5·(nlp_const + (x−μ)ᵀ·prec·(x−μ)) (negative_log_posterior); g or nlp may be NULL. */
int hmcx_mvn_eval(hmcx_ctx* ctx, int dim, int C, const double* mu, const double* prec, double nlp_const,
                  const double* x, double* g, double* nlp);

/* ------------------------------------------------------------------ full-batch HMC, linear models
 * Replaces cpu/hmc.py:39-64 (step) with the softmax (models/cpu/softmax.py) or logistic
 * (models/cpu/logistic.py) model, one chain: per step, momentum p ~ N(0,1) (hmc.py:41, draw order
 * weights then bias), then for it < n_iter, per var v in (weights, bias):
 *   p_v −= (½ε)·g_v;  q_v += ε·p_v;  g = grad(q);  p_v −= ε·g_v          (hmc.py:49-54)
 * with g = grad(q0) before the loop (hmc.py:47), p ← −p, and the MH accept
 * A = min(1, exp(E_cur − E_new)), E = nlp + ½Σp² (hmc.py:56-79; nlp = −(ll + log_prior)/N).
 * The whole schedule runs on the device: per gradient one k_fwd + one k_grad launch with the
 * kick/drift fused into the gradient epilogue; energies, accept and commit in step kernels.
 * log_prior: softmax — the constant `log_prior` (softmax.py:22-30); logistic — Σ_var
 * (lp_const[var] − ½·alpha·Σθ_var²) with Σθ² on the device (logistic.py:15-21).
 * X [N][D] (full batch: B = N rows), Y [N][K] one-hot (softmax) or [N] 0/1 (logistic, K = 1).
 * Noise as hmcx_sampler_args (BUFFER: noise_off[s], P = D·K + K momentum normals per step). */
typedef struct hmcx_hmc_args {
  int dtype;
  int model;               /* HMCX_MODEL_SOFTMAX or HMCX_MODEL_LOGISTIC                  */
  int B, D, K, n_steps;    /* B = N (full batch)                                        */
  double alpha;
  double log_prior;        /* softmax: constant log prior                               */
  double lp_const[2];      /* logistic: dim·½·log(alpha/2π) of weights, bias            */
  const void* X;
  const void* Y;
  const double* eps;       /* host [n_steps]                                            */
  const int32_t* n_iter;   /* host [n_steps]  max(0, L − 1)                            */
  const double* u_accept;  /* host [n_steps]                                            */
  int noise_mode;
  const double* noise;     /* device, BUFFER                                            */
  const int64_t* noise_off;/* host [n_steps], BUFFER                                    */
  uint64_t seed;
  uint32_t chain, step_base;
  void* W;                 /* device [D][K] state, updated in place                     */
  void* b;                 /* device [K]                                                */
  double* out_A;           /* device [n_steps]                                          */
  int32_t* out_accepted;   /* device [n_steps]                                          */
  double* out_nlp;         /* device [n_steps]: nlp of the state kept after step s     */
  double* out_E;           /* device [n_steps*2] (E_current, E_new) or NULL             */
  void* out_trace;         /* device [n_steps][D*K+K] (dtype) or NULL: state after s    */
  void* out_mom;           /* device [n_steps][D*K+K] (dtype) or NULL: momentum drawn   */
} hmcx_hmc_args;
int hmcx_hmc_run(hmcx_ctx* ctx, const hmcx_hmc_args* a);

/* Leapfrog arithmetic on device vectors of n elements (dtype), for hmc.step on models without a
 * fused entry (the MLP): mode 0  y −= a·x;  mode 1  y += a·x  (hmc.py:50-53, p −= ε·g, q += ε·p).
 * hmcx_sumsq gives the kinetic energy's Σp² (hmc.py:74-79). */
int hmcx_axpy(hmcx_ctx* ctx, int dtype, int mode, int64_t n, double a, const void* x, void* y);

/* ------------------------------------------------------------------ MLP model (config 3)
 * Replaces hamiltonian/models/gpu/mlp.py:19-31 (MyNetwork: l1 -> relu(dropout) -> l2 ->
 * relu(dropout) -> dropout -> l3) and :47-82 (grad / log_likelihood / negative_log_posterior)
 * without Chainer.  Parameters in Chainer's layout, L.Linear W = [out][in]:
 *   W1 [n_mid][n_in], b1 [n_mid], W2 [n_mid][n_mid], b2 [n_mid], W3 [n_out][n_mid], b3 [n_out].
 * Dropout (mlp.py:29-31, ratio 0.1, train mode): mask = (u >= 0.1) / 0.9 for the three [B][n_mid]
 * activations of every forward.  mask_mode BUFFER: masks[...] holds them (3·B·n_mid values per
 * forward, dtype); PHILOX: u = Philox(seed, chain, step, slot = forward index, element).       */
typedef struct hmcx_mlp_params {
  void* p[6];              /* W1, b1, W2, b2, W3, b3 (device, dtype) */
} hmcx_mlp_params;

/* Philox dropout masks of one forward: out [3][B][n_mid] (dtype) = (u >= 0.1)/0.9 with
 * u = Philox(seed, chain, step, slot, element) — the masks hmcx_mlp_sghmc_run draws (PHILOX). */
int hmcx_mlp_masks(hmcx_ctx* ctx, int dtype, int B, int n_mid, uint64_t seed, uint32_t chain, uint32_t step,
                   uint32_t slot, void* out);

/* grad = ∇ mean softmax-CE(net(X), y) + ½·alpha·θ for all six parameters (mlp.py:47-64).
 * y: device int32 [B] labels.  masks: device [3][B][n_mid] or NULL (no dropout).
 * grads: output pointers, same shapes.  loss (device double[1] or NULL): the mean CE. */
int hmcx_mlp_grad(hmcx_ctx* ctx, int dtype, const void* X, const int32_t* y, int B, int n_in, int n_mid,
                  int n_out, const hmcx_mlp_params* par, const void* masks, double alpha,
                  hmcx_mlp_params* grads, double* loss);

/* loss = mean softmax-CE (mlp.py:66-78 returns the loss); logits [B][n_out] optional output
 * (predict, mlp.py:84-96). */
int hmcx_mlp_loss(hmcx_ctx* ctx, int dtype, const void* X, const int32_t* y, int B, int n_in, int n_mid,
                  int n_out, const hmcx_mlp_params* par, const void* masks, double* loss, void* logits);

/* SGHMC steps for the MLP (reference cpu/sghmc.py:19-39 with the A1 completion; energies from
 * mlp.py:80-82 nlp = loss + log_prior, log_prior = −Σ_var ½·alpha·Σθ²/dim).  Sub-steps follow
 * order[0..5] (canonical indices 0=W1 1=b1 2=W2 3=b2 4=W3 5=b3 in the caller's start_p order).
 * Noise BUFFER: per step, normals in the reference's draw order — momentum of every variable
 * in `order`, then per leapfrog iteration one draw per variable in `order` — from noise_off[s].
 * PHILOX: slot 0 momentum, slot it+1 iteration it, element = offset of the variable in `order`
 * + index.  Masks: forward f of step s (f = 0 .. 6·n_iter−1 for the gradient calls, then the
 * proposal's and the current state's energies) — BUFFER: masks + mask_off[s] + f·3·B·n_mid;
 * PHILOX: slot 0x80000000 + f.  out_loss[s] = mean CE loss (log_likelihood, mlp.py:66-78) and out_nlp[s] =
 * loss + log_prior (negative_log_posterior) of the state kept after step s, both under the masks
 * of that state's energy forward. */
typedef struct hmcx_mlp_sghmc_args {
  int dtype;
  int B, n_in, n_mid, n_out, n_steps;
  int order[6];
  double alpha;
  const void* X;           /* device [N][n_in] */
  const int32_t* y;        /* device [N] labels */
  const int64_t* row0;     /* host [n_steps] */
  const double* eps;       /* host [n_steps] */
  const int32_t* n_iter;   /* host [n_steps] */
  const double* u_accept;  /* host [n_steps] */
  int noise_mode;
  const double* noise;     /* device, BUFFER */
  const int64_t* noise_off;/* host [n_steps], BUFFER */
  int mask_mode;
  const void* masks;       /* device, BUFFER (dtype) */
  const int64_t* mask_off; /* host [n_steps], BUFFER */
  uint64_t seed;
  uint32_t chain, step_base;
  hmcx_mlp_params par;     /* state, updated in place */
  double* out_A;           /* device [n_steps] */
  int32_t* out_accepted;   /* device [n_steps] */
  double* out_loss;        /* device [n_steps] */
  double* out_nlp;         /* device [n_steps] or NULL */
  double* out_E;           /* device [n_steps*2] (E_current, E_new) or NULL */
  int32_t* out_abort;      /* device [1] or NULL: the call's verdict — 1 when an exchange of the fused
                              layer-2/3 launches timed out; the state and every output of the call are
                              then invalid: restore the state and re-run with hmcx_set_mlp_fuse(ctx, 0).
                              NULL: the call waits for its stream and returns an error instead. */
} hmcx_mlp_sghmc_args;
int hmcx_mlp_sghmc_run(hmcx_ctx* ctx, const hmcx_mlp_sghmc_args* a);

/* Full-batch HMC leapfrog trajectory of the MLP in one call: replaces the per-variable loop of
 * hamiltonian/inference/cpu/hmc.py:46-56 as the GPU hmc.step runs it on the MLP (the reference's
 * gpu/hmc.py step with models/gpu/mlp.py grad).  With g = grad(q) first, per iteration and per
 * variable v in order[0..5]:  p_v −= ε/2·g_v;  q_v += ε·p_v;  g = grad(q);  p_v −= ε·g_v  (hmc.py:50-53),
 * then p = −p (hmc.py:55-56, as p − 2·p).  grad is hmcx_mlp_grad (∇ mean CE + ½·alpha·θ, all six
 * variables, 1 + 6·n_iter calls; every call but the last computes only the one or two components the
 * next kicks read, the last one all six); the kicks and drifts are hmcx_axpy's — the same kernels in
 * the same order as the host loop, so the trajectory is bit-identical to it.  Masks per gradient call:
 *   HMCX_MLP_MASKS_NONE    no dropout;
 *   HMCX_MLP_MASKS_FIXED   masks [3][B][n_mid] (dtype) for every call;
 *   HMCX_MLP_MASKS_PHILOX  call k draws hmcx_mlp_masks(seed, chain, step, slot0 + k) into masks (scratch).
 * q and p are advanced in place; g holds the gradient at the final position on return. */
#define HMCX_MLP_MASKS_NONE 0
#define HMCX_MLP_MASKS_FIXED 1
#define HMCX_MLP_MASKS_PHILOX 2
typedef struct hmcx_mlp_leapfrog_args {
  int dtype;
  int B, n_in, n_mid, n_out, n_iter;
  int order[6];            /* canonical variable indices 0=W1 .. 5=b3 in the caller's start order */
  double eps, alpha;
  const void* X;           /* device [B][n_in] */
  const int32_t* y;        /* device [B] labels */
  hmcx_mlp_params q, p, g; /* device: position, momentum (in/out), gradient (out) */
  int mask_mode;
  void* masks;             /* device [3][B][n_mid]: FIXED input / PHILOX scratch */
  uint64_t seed;
  uint32_t chain, step, slot0;
} hmcx_mlp_leapfrog_args;
int hmcx_mlp_hmc_leapfrog(hmcx_ctx* ctx, const hmcx_mlp_leapfrog_args* a);

/* on = 0: hmcx_mlp_sghmc_run stops fusing layer 2 and layer 3 into one launch (no cross-workgroup
 * exchange; one more launch per forward) — the recovery path after out_abort; on = 1 restores it. */
int hmcx_set_mlp_fuse(hmcx_ctx* ctx, int on);
/* Wide SGLD (config 5, hmcx_sgld_run with K ≤ 64 or several chains): fused forward + softmax (1, the
 * default) or the three-launch form (0).  A fused call given out_abort stores its verdict there
 * (stream-ordered, no host wait): 1 means a team round timed out and W / b (pW / pb) are invalid —
 * restore the start state and re-run the call with hmcx_set_sgld_fuse(ctx, 0).  Without out_abort the
 * call restores and re-runs itself and waits for its stream (hmcx_get_recoveries counts either re-run
 * once the caller reports its own with hmcx_note_recovery). */
int hmcx_set_sgld_fuse(hmcx_ctx* ctx, int on);

/* ------------------------------------------------------------------ cross-rank gather (RCCL)
 * Replaces the reference's multi-chain result collection (hamiltonian/inference/cpu/
 * sghmc_multicore.py:86-94: Pool.map of per-worker posteriors, concatenated on the parent;
 * SURVEY §8(e)): one process per GPU samples its own chains with no communication, then ONE
 * all-gather over RCCL (xGMI) moves every rank's per-chain summaries (per-parameter Welford mean /
 * M2 and a thinned trace, packed by the caller) to every rank.  The communicator is created here
 * from a unique id that rank 0 makes (hmcx_comm_unique_id) and the launcher hands to every rank
 * (any out-of-band channel: the bench uses the torch.distributed gloo store).  Collectives run on
 * the context's stream and return once enqueued. */
typedef struct hmcx_comm hmcx_comm;
#define HMCX_COMM_ID_BYTES 128
int hmcx_comm_unique_id(void* id /* host [HMCX_COMM_ID_BYTES] */);
int hmcx_comm_init(hmcx_ctx* ctx, int nranks, int rank, const void* id /* host */, hmcx_comm** out);
int hmcx_comm_destroy(hmcx_comm* comm);
/* recv[r][0..count) = send of rank r (device doubles; recv holds nranks·count) */
int hmcx_allgather_chain_stats(hmcx_ctx* ctx, hmcx_comm* comm, const double* send, double* recv, uint64_t count);
/* recv = elementwise sum (op 0) or max (op 1) over the ranks of send (device doubles): the bench's
 * leapfrog total and max-over-ranks time */
int hmcx_allreduce_f64(hmcx_ctx* ctx, hmcx_comm* comm, const double* send, double* recv, uint64_t count, int op);

/* Cross-chain convergence diagnostics on the device (the reference has none — its
 * multi-chain layer concatenates posteriors, hamiltonian/inference/cpu/sghmc_multicore.py:86-94,
 * read back by hmc.py:132-138 backend_mean).  Per parameter p < P of C chains:
 *   out[p]       R̂ from per-chain moments (means / M2 [C][P] over n_moments draws; NaN when means
 *                is NULL),
 *   out[P + p]   split-R̂ of the traces (chains halved: 2C sequences of T/2 draws),
 *   out[2P + p]  bulk ESS (Geyer's initial monotone sequence on the split sequences),
 * with the definitions of dropout_hamiltonian_montecarlo_amd/diagnostics.py (BDA3 §11.4-11.5).
 * trace: device [C][T][P] float64 (T >= 4) — e.g. the buffer hmcx_allgather_chain_stats filled;
 * means, M2, out: device float64.  Stream-ordered; returns before the kernel completes. */
int hmcx_chain_diagnostics(hmcx_ctx* ctx, int C, int T, int P, const double* trace, const double* means,
                           const double* M2, int64_t n_moments, double* out);

#ifdef __cplusplus
}
#endif
#endif /* HMCX_H */
