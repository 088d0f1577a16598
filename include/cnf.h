/*
 * cnf.h — C ABI of libcnf_hip.so, the MI355X (gfx950) implementation of the
 * conditional-RealNVP forward / inverse + Jacobian log-det hot path of
 * USArmyResearchLab/ARL_Conditional_Normalizing_Flows.
 *
 * The reference is pure TensorFlow/Keras Python and has no FFI of its own; the
 * interfaces replaced are its Python layer/model protocol, and every entry point
 * below cites the reference function it stands in for
 * (file:line into conv_cINN_make_model.py unless stated).
 *
 * Conventions
 *   - All tensors are device pointers, NHWC, fp32, batch-first, contiguous.
 *   - The caller allocates ALL device memory (params, activations, workspace);
 *     the library never frees caller pointers. A plan owns only small constant
 *     tables (index maps) that it uploads once, lazily, on first use.
 *   - Every compute call is asynchronous on the given stream (a hipStream_t passed
 *     as void*; NULL = default stream) and may be captured into a hipGraph.
 *   - Return value: 0 = OK, negative = error class (CNF_E_*); the message is
 *     available from cnf_last_error() (thread-local). No C++ exception crosses
 *     the ABI. A plan is not thread-safe: one host thread per plan, one process
 *     per GPU.
 *   - Reductions are deterministic (no float atomics): repeated runs are bitwise
 *     identical.
 */
#ifndef CNF_H_
#define CNF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CNF_OK 0
#define CNF_E_INVALID (-1)   /* bad argument / shape: the reference's AssertionError */
#define CNF_E_HIP (-2)       /* HIP runtime error */
#define CNF_E_STATE (-3)     /* call out of order / unsupported configuration */

#define CNF_GROUP_REFERENCE 0 /* late-bound Lambda closure: every group reads the last slice
                                 (conv_cINN_base_functions.py:402) — the reference's behaviour */
#define CNF_GROUP_INTENDED 1  /* textbook grouped conv: group j reads slice j */

#define CNF_LAYER_COUPLING 0
#define CNF_LAYER_SQUEEZE 1
#define CNF_LAYER_FACTOR 2

typedef struct cnf_plan cnf_plan;

/* Constructor arguments of cFlow.__init__ (conv_cINN_make_model.py:1431-1442). */
typedef struct cnf_flow_desc {
    int io_h, io_w, io_d;                 /* io_shape */
    int x_d;                              /* depth of x inside xy */
    int num_blocks;                       /* len(squeeze_factor_block_list) */
    const int* squeeze_factor_block_list; /* [num_blocks], entries 0/1 */
    const int* resnext_block_list;        /* [num_blocks] */
    const int* num_kernels_list;          /* [num_blocks] */
    const int* cardinality_list;          /* [num_blocks] */
    float lambda_y;                       /* default 100 */
    int ksize;                            /* default 3 (only 3 is implemented on GPU) */
    int layer_norm;                       /* LAYER_NORM, default 1 */
    int dilations;                        /* DILATIONS, default 1 */
    int group_mode;                       /* CNF_GROUP_* (default REFERENCE) */
    /* Debug options, NULL or "" for the defaults (what is benchmarked): "NAME=V[,NAME=V...]" selecting
     * the alternative code paths the parity tests compare against — NETLDS, GC, PW, GENERIC, LAYOUT,
     * FUSE_COUPLING, LDS_BWD, TRAIN_ALT, TRAIN_SCHED (meanings: csrc/cnf_kernels.h Options). Parsed at
     * cnf_plan_create (unknown name: CNF_E_INVALID); the string is not kept. Without a GENERIC entry, a
     * flow on images of 64 x 64 and above runs the generic k_pw / k_gc kernels (GENERIC=6; the
     * shape-specialised ones showed intermittent differences there). The library reads no
     * environment variable. No reference counterpart (the Keras model has no such switches). */
    const char* debug_options;
} cnf_flow_desc;

/* One entry of cFlow.layers_list (conv_cINN_make_model.py:1630-1689). */
typedef struct cnf_layer_info {
    int kind;              /* CNF_LAYER_* */
    int coupling_index;    /* ordinal among coupling layers, -1 otherwise */
    int block;             /* coupling block */
    int h, w, d;           /* io shape of the block (in_shape of the layer) */
    int mask;              /* which_mask 0..3 (coupling) */
    int hc, wc, dc1, dc2;  /* compressed u1c shape / uv2_d (coupling) */
    int num_kernels;       /* halved for checkerboard masks (:420-423) */
    int cardinality;
    int num_res_blocks;
    int num_dilations;
    int dilations[8];
    int num_prev_factors;  /* factor layers (:230-240) */
    int fused_net;         /* 1: both s,t nets run as one workgroup per image (k_net_lds) */
} cnf_layer_info;

/* Plan = cFlow.__init__ (:1431-1695): asserts, scale schedule, dilation
 * schedule, layer list, canonical parameter table. Host-only, no GPU work. */
int cnf_plan_create(const cnf_flow_desc* desc, cnf_plan** out);
void cnf_plan_destroy(cnf_plan* plan);

int cnf_plan_num_layers(const cnf_plan* plan);
int cnf_plan_layer_info(const cnf_plan* plan, int layer, cnf_layer_info* out);

/* Canonical parameters: one flat fp32 vector, tensors in Keras order (net A,
 * then net b, per coupling layer; Conv2D kernels HWIO, LayerNormalization
 * gamma/beta over the flattened H*W*C axis). */
int64_t cnf_plan_num_params(const cnf_plan* plan);
int cnf_plan_num_param_tensors(const cnf_plan* plan);
int cnf_plan_param_tensor(const cnf_plan* plan, int index, char* name, int name_cap,
                          int64_t* offset, int* ndim, int shape[4]);

/* Device-side auxiliary parameter image (every conv's weights in its kernel's
 * staging layout, the grouped convs as dense images built from the per-group
 * Conv2D kernels, and the streamed layers' LN2 / LN3 gamma/beta gathered into
 * their t1 / t2 sub-tensor layouts). Size in floats; filled by cnf_pack_params,
 * which must run again whenever the canonical params change. */
int64_t cnf_plan_aux_floats(const cnf_plan* plan);
int cnf_pack_params(cnf_plan* plan, const float* params, float* aux, void* stream);

/* Workspace bytes for a batch of B images (all activations, LN-stat partials,
 * log-det partials). */
size_t cnf_plan_workspace_bytes(const cnf_plan* plan, int B);

/* cFlow.call(xy, direction=+1) (:1743-1772): xy[B,H,W,D] -> zy[B,H,W,D] in xy
 * layout, logdet_per_image[B] = sum over coupling layers of sum_{h,w,c} A(u1)
 * (the reference returns its batch mean, :1323-1326). xy and zy must not alias
 * (CNF_E_INVALID): the reference returns new tensors, and the fused schedule
 * reads xy after zy's first writes. */
int cnf_flow_forward(cnf_plan* plan, const float* params, const float* aux,
                     const float* xy, float* zy, float* logdet_per_image,
                     void* workspace, int B, void* stream);

/* cnf_flow_forward of the input as the reference's training pipeline prepares it
 * (conv_cINN.py:246-315): with logit_a in (0, 0.5) the logit map of
 * preprocess_dataset_class(LOGITS=True, a=logit_a) on the x channels
 * (conv_cINN_base_functions.py:174-231; 0: none), then instance_noise(., alpha) on every
 * channel (:635-654, the pipeline's 2 % noise: alpha = 0.98). xy_noisy[B,H,W,D] receives the
 * prepared input -- bit for bit cnf_logit (x channels) followed by cnf_instance_noise(.,
 * xy_noisy, B*H*W*D, alpha, seed, offset) -- and zy / logdet_per_image are cnf_flow_forward
 * of it. The preparation runs inside the first coupling layer's gather (no pass over xy)
 * when that layer is LDS-resident, otherwise as one pass first. xy_noisy is the xy of the
 * matching cnf_nll call. No two of xy, xy_noisy, zy may alias. */
int cnf_flow_forward_noise(cnf_plan* plan, const float* params, const float* aux,
                           const float* xy, float logit_a, float alpha, uint64_t seed,
                           uint64_t offset, float* xy_noisy, float* zy, float* logdet_per_image,
                           void* workspace, int B, void* stream);

/* cFlow.call(zy, direction=-1) (:1774-1798): zy -> xy (must not alias). */
int cnf_flow_inverse(cnf_plan* plan, const float* params, const float* aux,
                     const float* zy, float* xy, void* workspace, int B, void* stream);

/* coupling_layer.forward_and_Jacobian (:1258-1328) for layer `layer` of
 * layers_list: u -> v (shape of the layer's in_shape); logdet_accum[B] +=
 * per-image sum of A(u1) (pass NULL to skip). u and v must not alias. */
int cnf_coupling_forward(cnf_plan* plan, int layer, const float* params, const float* aux,
                         const float* u, float* v, float* logdet_accum,
                         void* workspace, int B, void* stream);

/* coupling_layer.backward (:1333-1394): v -> u. */
int cnf_coupling_inverse(cnf_plan* plan, int layer, const float* params, const float* aux,
                         const float* v, float* u, void* workspace, int B, void* stream);

/* squeeze_layer (:155-217): dir=+1 space_to_depth(2) in TF channel order,
 * dir=-1 depth_to_space(2). in: [B,H,W,C] (dir=+1) or [B,H,W,4C'] (dir=-1). */
int cnf_squeeze(const float* in, float* out, int B, int H, int W, int C, int dir, void* stream);

/* Channel-window copy used by factor_out_zy_layer (:256-329):
 * out[b,p,out_off + c] = in[b,p,in_off + c] for c < C, p < HW. */
int cnf_channel_copy(const float* in, int in_cs, int in_off, float* out, int out_cs, int out_off,
                     int C, int B, int HW, void* stream);

/* cFlow.log_loss terms (:1815-1848). per_image[B*3] = (llz, lly, logdet) with
 * llz = sum_{h,w} log N(z; 0, I_{x_d}), lly = -lambda_y * sum |y - y'|;
 * sums[4] = (sum_i loss_i, sum_i -llz_i, sum_i -lly_i, sum_i -logdet_i),
 * loss_i = -(llz_i + lly_i + logdet_i). Dividing sums by the (global) batch
 * gives the reference's (loss, z_loss, y_loss, detJ_loss). One kernel launch;
 * its last workgroup is found through a completion counter the plan keeps per
 * stream, so calls on different streams may run concurrently. 64 counters per
 * plan: a 65th stream reuses the least recently used one, its launch ordered
 * after that counter's last launch (a stream wait, no host wait; inside graph
 * capture that slot needs one earlier uncaptured call). The first call on a plan uploads its tables (not capturable:
 * cnf_pack_params does the same, call it before graph capture). */
int cnf_nll(const cnf_plan* plan, const float* xy, const float* zy, const float* logdet_per_image,
            float* per_image, float* sums, int B, void* stream);

/* ---------------------------------------------------------------------------
 * NLL training step (cFlow.train_step, :1850-1880: GradientTape over log_loss,
 * then Adam). Replaces the TF autodiff of the whole log_loss graph.
 * ------------------------------------------------------------------------- */

/* Training workspace bytes for B images (the inference workspace, the saved
 * coupling-layer inputs, one layer's recomputed activations, gradient buffers). */
size_t cnf_plan_train_workspace_bytes(const cnf_plan* plan, int B);

/* cnf_flow_forward that also saves every coupling layer's input into
 * train_workspace (for cnf_flow_backward on the same xy / zy). */
int cnf_flow_forward_train(cnf_plan* plan, const float* params, const float* aux,
                           const float* xy, float* zy, float* logdet_per_image,
                           void* train_workspace, int B, void* stream);

/* dparams[num_params] = d loss / d params for this shard, where
 * loss = -(sum_i (llz_i + lly_i + logdet_i)) * inv_batch (inv_batch = 1 / global
 * batch size: summing dparams over data-parallel shards gives the gradient of the
 * reference's batch-mean loss). d|y - y'| / dy = sign(y - y') (0 at 0), as TF. */
int cnf_flow_backward(cnf_plan* plan, const float* params, const float* xy, const float* zy,
                      void* train_workspace, int B, float inv_batch, float* dparams, void* stream);

/* cnf_flow_backward for data-parallel training with the gradient reduction
 * overlapped (conv_cINN_make_model.py:1863-1870):
 *  - global_count (device, 1 float) is the global image count, e.g. red5[4] of
 *    cnf_nll_allreduce: inv_batch = 1 / *global_count is taken on the device, so
 *    no host read of the all-reduced count sits between forward and backward;
 *  - layer_done (may be NULL) is called on the calling host thread as soon as the
 *    launches producing coupling layer `coupling_index`'s parameter gradients
 *    (names "c<index>.*", one contiguous range of dparams) are enqueued on
 *    `stream` (the backward's side streams have joined it). Work the callback
 *    enqueues behind that point on `stream` (or on a stream waiting for it), e.g.
 *    cnf_allreduce_sum_f32 of that range, overlaps the backward of the layers
 *    before it. Every coupling layer is reported exactly once, in an order that is
 *    the same on every rank: reverse index order, except that a layer whose
 *    weight gradients run on a side stream (the split LDS-layer backward) is
 *    reported when the stream first waits for them, two such layers later. */
typedef void (*cnf_layer_done_fn)(void* user, int coupling_index);
int cnf_flow_backward_ex(cnf_plan* plan, const float* params, const float* xy, const float* zy,
                         void* train_workspace, int B, const float* global_count, float* dparams,
                         cnf_layer_done_fn layer_done, void* user, void* stream);

/* Backward of one coupling layer (layer index into layers_list) at input u:
 * du = dL/du and dparams = dL/dparams (zeroed first; only this layer's entries
 * are non-zero) for upstream dv = dL/dv and dlogdet = dL/d(per-image log-det). */
int cnf_coupling_backward(cnf_plan* plan, int layer, const float* params, const float* u,
                          const float* dv, float* du, float dlogdet, void* train_workspace,
                          int B, float* dparams, void* stream);

/* Keras Adam (conv_cINN.py:567 Adam(3e-4); keras defaults beta_1 0.9, beta_2 0.999,
 * epsilon 1e-7): m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
 * p -= lr sqrt(1 - b2^t) / (1 - b1^t) * m / (sqrt(v) + eps), t = step >= 1. */
int cnf_adam_step(float* params, const float* grads, float* m, float* v, int64_t n, float lr,
                  float beta_1, float beta_2, float epsilon, int step, void* stream);

/* ---------------------------------------------------------------------------
 * TOYcINN (BASELINE configs[0]): the dense conditional flow of
 * TOYcINN_make_model.py:29-506 on 3-dimensional points.
 * ------------------------------------------------------------------------- */
typedef struct cnf_toy_desc {
    int io_shape;              /* must be 3 (the reference masks, :149-163) */
    int x_d;                   /* 1 or 2 */
    int num_coupling_layers;   /* <= 128 */
    int intermediate_dims;     /* H <= 64 */
    int num_layers;            /* hidden Dense layers after the first */
    const int* mask_indices;   /* [num_coupling_layers], a permutation (cINN_affine.mask_indices) */
    float lambda_y;            /* 100 in the reference */
} cnf_toy_desc;

/* Number of fp32 parameters: per network j (j = 0..L-1, mask type j % 6), the b net then the A
 * net, each Dense as kernel [in][out] then bias [out] (:48-94). */
int64_t cnf_toy_num_params(const cnf_toy_desc* d);

/* cINN_affine.call(u, direction) (:237-417): direction -1 = xy' -> zy (reverse layer order,
 * log_detJ[B] = per-sample sum of A), +1 = zy -> xy'. u, v: [B][3], must not alias.
 * per_sample[B*3] (direction -1, optional) = (llz, lly, log_detJ) of log_loss (:419-451). */
int cnf_toy_call(const cnf_toy_desc* d, const float* params, const float* u, float* v, float* log_detJ,
                 float* per_sample, int B, int direction, void* stream);

/* Batch sums of the toy log_loss terms: sums[4] = (sum loss_i, sum -llz_i, sum -lly_i,
 * sum -log_detJ_i); divide by B for the reference's 4-tuple. */
int cnf_toy_nll_sums(const float* per_sample, float* sums, int B, void* stream);

/* ---- input transforms (the step before the path; conv_cINN_base_functions.py) ----------- */

/* Logit preprocessing of preprocess_dataset_class(LOGITS=True) (:174-231), elementwise over n
 * values in [0, 1]: x -> (logit(a + (1-a) b x) - logit(a)) / (logit(1-a) - logit(a)),
 * b = (1-2a)/(1-a). inverse != 0 applies de_logitify (:287-318) instead. out may alias x. */
int cnf_logit(const float* x, float* out, int64_t n, float a, int inverse, void* stream);

/* Super-resolution preprocessing (preprocess_dataset_SR :233-279 with down/up :74-164):
 * hires [B][H][W][C] -> xy [B][H>>x_down][W>>x_down][2C] with x0 = down^x_down(hires),
 * y = up^y_levels(down^y_levels(x0)) (nested 2x2 means, then 2x2 repeats) and x = x0 - y when
 * residual (RESIDUAL=True), else x0; xy = concat(x, y). 'SR2,1': x_down 0, y_levels 1;
 * 'SR4,2': x_down 1, y_levels 1; the 4x / 8x benchmark configs: y_levels 2 / 3. H and W must be
 * divisible by 2^(x_down + y_levels). */
int cnf_sr_preprocess(const float* hires, float* xy, int B, int H, int W, int C, int x_down, int y_levels,
                      int residual, void* stream);

/* 2x2 average-pool down (:74-125) / 2x2 repeat up (:127-160) of [B][H][W][C]. */
int cnf_down(const float* in, float* out, int B, int H, int W, int C, void* stream);
int cnf_up(const float* in, float* out, int B, int H, int W, int C, void* stream);

/* instance_noise (:635-654): out = alpha x + (1 - alpha) N(0, 1), and renew_noise (:660-676)
 * with x == NULL: out = N(0, 1). Normals from a counter-based generator (Philox4x32-10 +
 * Box-Muller): element i of a call depends only on (seed, offset + i), so results are
 * reproducible and independent of the launch shape. out may alias x. */
int cnf_instance_noise(const float* x, float* out, int64_t n, float alpha, uint64_t seed, uint64_t offset,
                       void* stream);

/* ---------------------------------------------------------------------------
 * Data-parallel exchange: one process per GPU, the batch
 * sharded over ranks, ONE all-reduce of the NLL sums. Replaces the batch means
 * of the log-det (:1323-1326) and of log_loss (:1840-1848) over a sharded batch.
 * RCCL over xGMI, loaded at run time (CNF_E_STATE when librccl is absent).
 * ------------------------------------------------------------------------- */
#define CNF_COMM_ID_BYTES 128
typedef struct cnf_comm cnf_comm;

/* Rank 0 creates the communicator id and hands it to every rank by any
 * out-of-band means (a file, a key-value store, MPI). */
int cnf_comm_unique_id(char uid[CNF_COMM_ID_BYTES]);
/* Collective over `world` processes; binds the communicator to the calling
 * thread's current HIP device. */
int cnf_comm_init(int rank, int world, const char uid[CNF_COMM_ID_BYTES], cnf_comm** out);
void cnf_comm_destroy(cnf_comm* comm);
/* In-place sum all-reduce of n fp32 device values, asynchronous on stream. */
int cnf_allreduce_sum_f32(cnf_comm* comm, float* buf, size_t n, void* stream);
/* The path's exchange step: red5 (device, 5 floats) = sum over ranks of
 * (sums[0..3] of this rank's cnf_nll, B); red5[k] / red5[4] for k < 4 is the
 * reference's (loss, z_loss, y_loss, detJ_loss) over the global batch. comm may
 * be NULL (one process: no collective, red5 = local sums and B). */
int cnf_nll_allreduce(cnf_comm* comm, const float* sums, int B, float* red5, void* stream);

/* Plan introspection (tests): the canonical parameter index behind every float
 * of the kernel image (which = 0; -1 = zero padding; cnf_pack_params computes
 * aux[i] = params[map[i]]) or of the dense training image (which = 1: every
 * conv as [taps][cin][cout] + bias padded to 4, in layer order). Returns the
 * map length; copies min(length, cap) entries when out != NULL. */
int64_t cnf_plan_weight_map(const cnf_plan* plan, int which, int64_t* out, int64_t cap);

/* Measurement hooks (bench.py): number of kernel launches recorded by the last
 * forward/inverse call on this plan, their kernel symbol names, and a re-launch
 * of one recorded launch with identical arguments (same buffers). */
int cnf_plan_num_recorded_launches(const cnf_plan* plan);
int cnf_plan_recorded_launch_info(const cnf_plan* plan, int i, char* name, int name_cap,
                                  double* flops, double* bytes);
int cnf_plan_relaunch(cnf_plan* plan, int i, void* stream);
/* In-stream launch timing: while on, every kernel of a forward/inverse call is
 * dispatched with hipExtLaunchKernelGGL start/stop events, which receive the
 * kernel's own begin/end timestamps (eager calls only, not inside graph
 * capture); cnf_plan_launch_time_ms then gives launch i's GPU duration in its
 * place in the sequence (waits for it; 0 for a launch that is not a kernel). */
int cnf_plan_set_launch_timing(cnf_plan* plan, int on);
int cnf_plan_launch_time_ms(const cnf_plan* plan, int i, float* ms);

const char* cnf_last_error(void);
const char* cnf_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CNF_H_ */
