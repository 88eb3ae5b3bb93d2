// Launch-argument structs and host launcher declarations shared by the HIP kernel translation
// units and the PyTorch bindings.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

namespace dfa {
typedef __bf16 bf16;
}

namespace dfa {

enum { MODE_DIRECT = 0, MODE_FWD = 1, MODE_DGRAD = 2 };

// Dropout folded into a producer's epilogue (same mask as csrc/layers.hip dropout_kernel: element i of
// the produced tensor is kept when hash(seed ^ step * 0x9E3779B1, i) >= thresh, kept values * scale)
struct DropSpec {
  int on;
  unsigned thresh;  // p * 2^32
  float p, scale;   // scale = 1 / (1 - p)
  unsigned long long seed;
  const long long* step;  // device step counter (nullable)
  int step_add;           // masks use step[0] + step_add (1 when the counter advances at the END of a step)
};
inline DropSpec make_drop(float p, unsigned long long seed, const long long* step, int step_add = 0) {
  DropSpec d{};
  if (p > 0.f) {
    d.on = 1;
    d.thresh = (unsigned)((double)p * 4294967296.0);
    d.p = p;
    d.scale = 1.f / (1.f - p);
    d.seed = seed;
    d.step = step;
    d.step_add = step_add;
  }
  return d;
}

// BatchNorm statistics emitted by the PRODUCING conv launch (csrc/bn_epi.h): every row tile reduces the
// values it stored into a partial [2][N] row, and the launch's last arrivers (two fixed-order levels)
// finalise them, so the BatchNorm that consumes the output needs neither a statistics pass over it nor a
// finalize launch.  mode 0 (forward): sums of y and y^2 -> mean, invstd, running statistics.  mode 1
// (backward, the conv producing the BN's output gradient g, relu' already applied): sums of g and
// g * xhat with xhat = (x - mean) * invstd of the BN input x -> dgamma, dbeta and the coefficients of
// dx = k1 g + k2 x + k3 (bn_dx).
struct BnEpi {
  float* part;        // [ntm][2][N] row-tile partials (write-through), then [ngrp][2][N] group partials
  unsigned* ticket;   // [ncolgroups][1 + ngrp] arrival tickets, zero between launches (last arrivers re-arm)
  int ntm, ngrp;      // row tiles of the launch, groups of 16 of them
  int mode;
  const bf16* x;                         // mode 1: the BN input [M][ldc]
  const float *mean, *invstd, *gamma;    // mode 1 inputs (forward statistics, scale)
  float *mean_out, *invstd_out, *run_mean, *run_var;  // mode 0 outputs
  float *dgamma, *dbeta, *coef;          // mode 1 outputs (coef [3][N])
  float momentum, eps, gscale;
};

// BatchNorm statistics accumulated in the PRODUCING kernel's epilogue (csrc/bn_acc.h): every workgroup
// reduces the values it stored, per channel and in a fixed order, and adds them in fp64 into replica
// (blockIdx % nrep) of `acc` (no ticket, no wait: the adds are fire-and-forget); the consuming pass
// (bn_apply_acc / bn_dx_acc, csrc/bn.hip) finalises them in its prologue.  mode 0 (forward): [S = sum y,
// Q = sum y^2]; mode 1 (backward, relu' already applied to the stored g): [S = sum g, Q = sum g * xhat],
// xhat = (x - mean) * invstd of the BN input x -- for up to two BatchNorms that share g (a ResNet block's
// bn2 and its projection BN read the same block-output gradient).  fp64 adds of fixed-order fp32
// partials: the sums depend on arrival order only in the last bits of a double.
struct BnAcc {
  double* acc;       // [nrep][2][N] (nullptr: off)
  double* acc2;      // mode 1: the second BatchNorm's [nrep][2][N] (nullptr: none)
  const bf16* x;     // mode 1: BN input [M][ldc] at the output's positions
  const float *mean, *invstd;
  const bf16* x2;    // mode 1: the second BatchNorm's input
  const float *mean2, *invstd2;
  int nrep, mode;
};
constexpr int kBnAccMaxRep = 16;

struct IGemmArgs {
  const bf16* src;   // A source: [M][lda] (direct) or NHWC [B][SH][SW][SC] (conv gathers)
  const bf16* w;     // [Npad16][Kpad32] bf16, zero padded
  const float* bias; // [N] or nullptr
  const bf16* mask;  // [M][ldc] producer activation for relu' (nullptr = none)
  const bf16* res;     // [M][ldc] residual added before relu / mask (nullptr = none): ResNet shortcut gradient
  const bf16* resmask; // [M][ldc] res counts only where resmask > 0 (nullptr = everywhere)
  void* out;         // [M][ldc] bf16 or fp32
  int M, N, K, Kpad, lda, ldc;
  int SH, SW, SC, OH, OW, KH, KW, stride, pad;
  int stride_w, pad_w;  // column stride / left padding (stride, pad: row stride / top padding)
  int irregular;        // 1: KH != KW, stride_w != stride, pad_w != pad or asymmetric (Keras 'same') padding --
                        // only the generic kernels (igemm.hip) take such a geometry
  int relu, out_f32;
  float alpha;
  float* splitk_ws;  // igemm64 split-K partials [splits][M][N] (nullptr: no split)
  int splits;
  DropSpec drop;     // dropout after the activation (requires ldc == N, bf16 out)
  uint8_t* pool_code;  // conv forward + 2x2 max-pool (igemm64 POOL): out = pooled [M/4][N], code [M/4][N]
  BnEpi bn;            // BatchNorm statistics of the stored output, finalised inside the launch (bn.part
                       // != nullptr: igemm64, no split-K / pooling / parity-class launch)
  BnAcc bacc;          // BatchNorm statistics of the stored output accumulated by the epilogue (bacc.acc)
};

struct WgradArgs {
  const bf16* dy;     // [M][ldd]
  const bf16* src;    // activation (gather source, same conventions as IGemmArgs)
  float* partial;     // [splits][N][K+1] (splits > 1)
  float* gw;          // [N][K] final (splits == 1)
  float* gb;          // [N] final bias grad or nullptr
  int M, N, K, ldd, lda;
  int SH, SW, SC, OH, OW, KH, KW, stride, pad;
  int stride_w, pad_w, irregular;  // as IGemmArgs
  int m_per_split, splits, with_bias;
  float scale;
};

struct ParamDesc {
  long long off;      // offset into the fp32 master / grad / momentum flat buffers
  long long bf_off;   // offset of the bf16 [Npad][Kpad] copy (-1: vector param, no copy)
  long long bft_off;  // offset of the bf16 transposed dgrad copy (-1: none)
  int numel;
  int N, T, Ci;       // matrix view: [N][T*Ci]
  int block_start;    // first workgroup of this tensor
  int pad_;
};

// Small models: the descriptor table travels in the kernel arguments (scalar-cache reads instead of a
// dependent chain of global loads for the per-workgroup descriptor search).
constexpr int kInlineDescs = 32;
struct ParamDescTable {
  ParamDesc d[kInlineDescs];
};

hipError_t igemm_fwd(const IGemmArgs& a, int mode, hipStream_t st);
bool igemm_bacc_ok(const IGemmArgs& a, int mode);  // can the launch accumulate a.bacc (BatchNorm sums)
// 64-deep-step variant for the vectorizable cases (csrc/igemm64.hip); igemm_fwd dispatches to it
bool igemm64_supported(const IGemmArgs& a, int mode);
bool igemm64_pool_supported(const IGemmArgs& a);
// row tiles (= BatchNorm partial rows) of the igemm64 launch for this problem, 0 if it cannot emit them
int igemm64_bn_tiles(const IGemmArgs& a, int mode);
int igemm64_bn_layout(const IGemmArgs& a, int mode, int* ntn);
hipError_t bn_finalize_partials(const float* part, int ntm, int C, long long M, float* mean, float* invstd,
                                float* run_mean, float* run_var, float momentum, float eps, hipStream_t st);
// dY of a pooled conv from the pooled gradient and the argmax codes (NHWC, 2x2 windows)
hipError_t unpool2(const bf16* dyp, const uint8_t* code, bf16* dy, int B, int OH, int OW, int N, hipStream_t st);
hipError_t igemm64(const IGemmArgs& a, int mode, hipStream_t st);
// fp32 floats of split-K workspace igemm64 wants for this problem (0: no split); the caller allocates
// them and passes the buffer in IGemmArgs::splitk_ws
long long igemm64_splitk_floats(const IGemmArgs& a, int mode);
// out = epilogue(sum over a.splits of a.splitk_ws[s][M][N]) in a fixed order (igemm64's split-K combine)
hipError_t igemm64_splitk_combine(const IGemmArgs& a, hipStream_t st);
hipError_t igemm_wgrad(const WgradArgs& a, int mode, float* workspace, size_t ws_floats, hipStream_t st);
// conv weight gradient with transposed LDS reads (csrc/wgrad_tr.hip): conv, C % 8 == 0, no bias
bool wgrad_tr_supported(const WgradArgs& a, int mode);
hipError_t wgrad_tr(const WgradArgs& a, float* workspace, size_t ws_floats, hipStream_t st);
// 3x3 stride-1 pad-1 conv weight gradient, halo-tiled LDS staging (csrc/wgrad_halo.hip): C, N % 64 == 0
bool wgrad_halo_supported(const WgradArgs& a, int mode);
// 3x3 stride-1 pad-1 conv forward / data gradient, halo-tiled LDS staging (csrc/conv3_halo.hip)
bool conv3_halo_supported(const IGemmArgs& a, int mode);
hipError_t conv3_halo(const IGemmArgs& a, int mode, hipStream_t st);
hipError_t wgrad_halo(const WgradArgs& a, float* workspace, size_t ws_floats, hipStream_t st);
hipError_t maxpool_fwd(const bf16* x, bf16* y, int B, int H, int W, int C, int P, hipStream_t st,
                       DropSpec drop = DropSpec{});
hipError_t maxpool_bwd(const bf16* x, const bf16* dy, bf16* dx, int B, int H, int W, int C, int P, int relu_fused,
                       hipStream_t st);
hipError_t softmax_ce(const float* logits, const int* labels, bf16* dlogits, float* stats, int B, int C, int ldl,
                      int ldg, float grad_scale, hipStream_t st);
hipError_t dropout(const bf16* x, bf16* y, const bf16* mask, long long n, float p, unsigned long long seed,
                   const long long* step, hipStream_t st);
hipError_t gather_batch(const void* data, int data_is_u8, const int* labels, const long long* idx, bf16* out,
                        int* out_labels, int B, int row, float scale, long long nrows, hipStream_t st,
                        long long* step_inc = nullptr);
hipError_t gather_labels(const int* labels, const long long* idx, int* out, int B, long long nrows, hipStream_t st);
hipError_t add_act(const bf16* a, const bf16* b, bf16* out, long long n, int relu, hipStream_t st);
// Keras merge layers (csrc/merge.hip): out[rows][cout] from n inputs [rows][w[i]] (elementwise kinds: every
// w[i] == cout; Concatenate: the channels side by side, sum w[i] == cout).  merge_bwd writes grad[i] =
// d out / d in_i * dy for every input (Concatenate: the channel slice).
constexpr int kMergeMaxIn = 8;
constexpr int kMergeAdd = 0, kMergeSubtract = 1, kMergeMultiply = 2, kMergeAverage = 3, kMergeMaximum = 4,
              kMergeMinimum = 5, kMergeConcat = 6;
struct MergeArgs {
  const bf16* in[kMergeMaxIn];
  bf16* grad[kMergeMaxIn];
  const bf16* dy;
  bf16* out;
  int w[kMergeMaxIn];
  long long rows;
  int cout, n, kind;
};
hipError_t merge_fwd(const MergeArgs& a, hipStream_t st);
hipError_t merge_bwd(const MergeArgs& a, hipStream_t st);
hipError_t relu_bwd(const bf16* y, const bf16* dy, bf16* dx, long long n, hipStream_t st);
hipError_t gap_fwd(const bf16* x, bf16* y, int B, int HW, int C, hipStream_t st);
hipError_t gap_bwd(const bf16* dy, bf16* dx, int B, int HW, int C, hipStream_t st);
struct IndexStream {  // next-batch staging folded into the optimizer launch (csrc/optim.hip)
  const long long* src;  // [nsteps][B] batch indices
  long long* cursor;     // device step cursor
  long long* dst;        // [B] static index buffer read by the step
  int B, nsteps;
  // fused LeNet-5 conv-weight fragments rebuilt from the updated weights (csrc/lenet_frag.h); frag null = off
  void* frag;
  long long frag_w1, frag_w2;  // offsets of the conv1 / conv2 kernels in grad (and master / momentum)
  const float* snap;           // [2][2550] pre-update weights / momentum (lenet_reduce_kernel); read
                               // instead of master, which this same launch overwrites
  // device run statistics (callbacks / metrics without extra launches): the index-stream workgroup adds
  // this step's [loss sum, correct] to run_stats[0..1] and counts the applied update in run_stats[2]
  const float* step_stats;
  float* run_stats;
  // async PS, exclusive writer (csrc/async_ps.hip ps_excl_step): the update runs only when the admission
  // word *gate says accepted, and every new weight is also written to mirror (the rank's master shard)
  const unsigned* gate;
  float* mirror;
};
hipError_t sgd_multi(const ParamDesc* descs, int ndesc, int total_blocks, float* master, const float* grad,
                     float* mom_buf, bf16* wbf, const float* hyper, int apply_update, hipStream_t st,
                     const IndexStream* is = nullptr, const ParamDesc* host_descs = nullptr);
hipError_t sum_buffers(const float* const* ins, int nin, float* out, long long n, float scale, hipStream_t st);
hipError_t axpby(float* out, const float* a, const float* b, float alpha, float beta, long long n, hipStream_t st);
// ---- BatchNorm (csrc/bn.hip)
struct BnStatsArgs {
  const bf16* x;         // [M][C] BN input
  const bf16* mask;      // backward: g = dy * (mask > 0) (nullable)
  const bf16* dy;        // backward: incoming gradient
  const float* gamma;    // backward
  const float* mean;     // backward: saved batch statistics
  const float* invstd;
  float* mean_out;       // forward outputs
  float* invstd_out;
  float* run_mean;       // forward: running statistics (nullable)
  float* run_var;
  float* dgamma;         // backward outputs (flat gradient buffer slices)
  float* dbeta;
  float* coef;           // backward: [3][C] dx = k1*g + k2*x + k3
  float* ws;             // [G][2][C] partial slabs
  unsigned* counter;     // last-arriver ticket, 0 between launches
  int M, C;
  float momentum, eps, gscale;
};
struct BnApplyArgs {
  const bf16* x;
  bf16* y;
  const float *gamma, *beta, *mean, *invstd;      // eval: invstd holds the running variance
  const bf16* r;                                  // residual (nullable)
  const float *rgamma, *rbeta, *rmean, *rinvstd;  // BN of the residual (nullable: plain residual)
  int M, C, relu, eval;
  float eps;
};
int bn_stats_grid(int M, int C);
long long bn_stats_ws_floats(int M, int C);  // slabs + group slabs
int bn_stats_counters(int M, int C);         // ticket counters: 1 global + 1 per group of 16 workgroups
hipError_t bn_stats(const BnStatsArgs& a, int mode, hipStream_t st);  // mode 0 forward, 1 backward
hipError_t bn_apply(const BnApplyArgs& a, hipStream_t st);
hipError_t bn_dx(const bf16* x, const bf16* mask, const bf16* dy, bf16* dx, const float* coef, int M, int C,
                 hipStream_t st);
// statistics + apply (forward) / statistics + dx (backward) in one launch (C % 8 == 0, training mode);
// gen: a monotonically increasing generation word (any value to start, never reset)
bool bn_fused_ok(int C);
hipError_t bn_fwd_fused(const BnStatsArgs& a, const BnApplyArgs& p, unsigned* gen, hipStream_t st);
hipError_t bn_bwd_fused(const BnStatsArgs& a, bf16* dx, unsigned* gen, hipStream_t st);

// Consumers that finalise BnAcc sums in their prologue (csrc/bn.hip).  Every workgroup derives the
// per-channel coefficients from the replicas itself (fixed replica order, fp64); workgroup 0 also writes
// the finalised values (forward: mean, invstd, running statistics; backward: dgamma, dbeta, coef) and
// clears `zero` (this BatchNorm's accumulator of the OTHER direction, dead until the producer of the next
// step or pass refills it).
struct BnAccFin {
  const double* acc;  // [nrep][2][C]
  double* zero;       // [nrep][2][C] cleared by workgroup 0 (nullable)
  int nrep;
  float *mean, *invstd, *run_mean, *run_var;  // forward: outputs (run_* nullable); backward: mean/invstd in
  float momentum, eps;
  const float* gamma;                         // backward
  float *dgamma, *dbeta, *coef;               // backward outputs (coef [3][C], nullable)
  float gscale;
};
// y = act(bn(x) [+ r | + bn_r(r)]) with batch statistics from f (and fr: the residual's BatchNorm, RES 2)
hipError_t bn_apply_acc(const BnApplyArgs& a, const BnAccFin& f, const BnAccFin* fr, hipStream_t st);
// dx = k1 g + k2 x + k3 with the coefficients from f's backward sums (g: relu' already applied)
hipError_t bn_dx_acc(const bf16* x, const bf16* g, bf16* dx, const BnAccFin& f, int M, int C, hipStream_t st);
// dx[b][p][c] = dy[b][c] / HW * [mask > 0], with BatchNorm backward sums of dx (gap backward of ResNet)
hipError_t gap_bwd_bn(const bf16* dy, const bf16* mask, bf16* dx, int B, int HW, int C, const BnAcc& bacc,
                      hipStream_t st);

// fused Conv2D(+bias+ReLU)+MaxPool2x2 for small channel counts (convpool.hip)
// ---- fused dense head (csrc/mlphead.hip)
constexpr int kHeadMaxLayers = 4;
struct HeadLayer {
  const bf16* w;    // [Npad16][Kpad] compute copy
  const bf16* wt;   // dgrad layout [Kpad16][ldwt] (may be null for layer 0 when dX is not needed)
  const float* b;   // bias (nullable)
  float* gw;        // grad [N][K] fp32
  float* gb;        // bias grad (nullable)
  bf16* hT;         // H^T [N][ldt] (hidden layers)
  bf16* dzT;        // dZ^T [N][ldt]
  int K, N, Kpad, ldwt, tiles, pad_;
};
struct HeadArgs {
  HeadLayer L[kHeadMaxLayers];
  int nl, B, ldt, x_relu;
  const bf16* x;        // [B][K0] input activations
  bf16* xT;             // X^T [K0][ldt]
  bf16* dx;             // [B][K0] (nullable)
  float* logits;        // [B][C] fp32 (nullable)
  const int* labels;    // labels (indexed through idx when idx != null)
  const long long* idx;
  long long nrows;
  float grad_scale;     // d(loss)/d(logit) scale, 1/B for the mean
  float dx_scale;       // extra dX scale (a folded dropout's 1/(1-p); 0 = 1)
  float* loss_part;     // [nblocks][2]
  float* stats;         // [2] = (loss sum, correct)
  unsigned long long* stamps;  // profiling aid (head_set_stamps): per-block phase clocks, or null
  int nblocks, wg_tiles;
};
size_t head_train_lds(const HeadArgs& a);
hipError_t head_train(HeadArgs a, int phases, hipStream_t st);  // phases: 1 fwd/CE/bwd-data, 2 wgrad

void convpool_set_stamps(void* buf);  // [grid][32] uint64 s_memtime stamps, nullptr = off
// forward weight layout: [Npad16][Kpad2], column ky*RLp + kx*Cp + c (zero for c >= C) with
// RLp = round8(KW*Cp); pair layout (N <= 8): RLp = round8((KW+1)*Cp) and rows 8+n = row n shifted by Cp
void convpool_fwd_layout(int H, int W, int C, int KH, int KW, int pad, int N, int* Cp, int* Kpad2, int* pair);
void head_set_stamps(void* buf);
void convpool_dgrad_layout(int H, int W, int C, int KH, int KW, int pad, int N, int* pair, int* K2pad);
bool convpool_supported(int H, int W, int C, int KH, int KW, int pad, int N);
hipError_t convpool_fwd(const void* x, int x_u8, const long long* idx, long long nrows, float scale, int B, int H,
                        int W, int C, int KH, int KW, int pad, int N, const bf16* w, const float* bias, bf16* p,
                        uint8_t* code, hipStream_t st);
hipError_t convpool_wgrad(const void* x, int x_u8, const long long* idx, long long nrows, float scale, int B, int H,
                          int W, int C, int KH, int KW, int pad, int N, const bf16* dp, const uint8_t* code,
                          float* gw, float* gb, float* workspace, size_t ws_floats, hipStream_t st, int* deferred = nullptr);
hipError_t convpool_dgrad(const bf16* dp, const uint8_t* code, const bf16* wt, bf16* dx, int B, int H, int W, int C,
                          int KH, int KW, int pad, int N, hipStream_t st);
hipError_t slab_reduce(const float* partial, float* gw, float* gb, int N, int K, int Kt, int S, float scale,
                       hipStream_t st);
constexpr int kMaxSlabSegs = 8;
struct SlabSeg {
  const float* partial;  // [S][N][Kt]
  float* gw;             // [N][K]
  float* gb;             // [N] (column K) or nullptr
  int N, K, Kt, S, block0;
  float scale;
};
struct SlabSegs {
  SlabSeg s[kMaxSlabSegs];
  int n;
};
hipError_t slab_reduce_multi(SlabSegs segs, hipStream_t st);


// One-shot xGMI all-reduce (csrc/allreduce_p2p.hip).  Each rank's IPC buffer: flags
// [max_blocks][kP2PMaxRanks] u32 (flag_bytes, 4 KB aligned) followed by two staging halves of
// half_floats fp32 each.  Workgroup b always owns elements [b*kP2PChunk, (b+1)*kP2PChunk).
constexpr int kP2PMaxRanks = 8;
constexpr int kP2PChunk = 2048;
struct P2PArgs {
  char* bases[kP2PMaxRanks];  // bases[r] = rank r's buffer mapped into this process (bases[rank] local)
  float* data;                // in/out fp32 [n] (this rank's gradient, replaced by the sum * scale)
  long long n;
  unsigned* epochs;           // [max_blocks] per-block call counters (local)
  int* err;                   // sticky error word (local): bit 0 = a peer flag timed out
  int* herr;                  // host-mapped mirror of err (read by the host watchdog without a HIP call)
  long long flag_bytes, half_floats, timeout_ticks;  // timeout in wall_clock64 ticks (100 MHz)
  int rank, world, max_blocks;
  float scale;
};
hipError_t p2p_allreduce(const P2PArgs& a, hipStream_t st);

// In-kernel low-latency exchange (csrc/ll_exchange.h): 8-byte {fp32 value, u32 epoch} granules that a
// producing workgroup PUSHES into every peer's IPC-mapped region, so a reduction epilogue (the fused
// LeNet-5 reduce, ...) sums the W ranks' values of its own slot without a separate all-reduce launch.
// Region of rank r (inside its P2PComm allocation): [2 parities][nslots][kP2PMaxRanks src][kLLSlot].
constexpr int kLLSlot = 1024;  // granules per slot (one per thread of a 1024-thread epilogue)
constexpr int kLLParts = 8;    // owners a slot may be split over (LLComm::part_epochs)
struct LLComm {
  unsigned long long* bases[kP2PMaxRanks];  // bases[r] = rank r's LL region mapped into this process
  unsigned* epochs;                         // [nslots] per-slot call counters (local)
  unsigned* part_epochs;                    // [nslots][kLLParts] per-part counters (slots split over owners)
  int* err;                                 // sticky error word (shared with the P2P all-reduce)
  int* herr;                                // host-mapped mirror
  long long timeout_ticks;
  int rank, world, nslots;
};
// LL exchange self-test (csrc/allreduce_p2p.hip): out[slot][pos] = sum over ranks of in[slot][pos]
hipError_t ll_selftest(const LLComm& c, const float* in, float* out, int nslots, hipStream_t st);



// Device-resident async parameter server (csrc/async_ps.hip, protocol csrc/ps_device.h).  The fp32 master is
// SHARDED by contiguous parameter range: element i lives in shard i >> shard_shift, in that rank's HBM
// (IPC-mapped into every rank), so the appliers of different ranks update different shards -- and, inside a
// shard, different elements -- in parallel with lock-free per-element compare-and-swap adds (or plain
// read-modify-writes when this rank is the only writer).  The admitted-gradient version counter `ver`,
// the FCFS cursor and the completion arrays live in the server rank's control buffer; `ver` advances by
// a lock-free CAS whose check is the staleness bound.  No lock is ever held across an apply.
struct PSArgs {
  unsigned* ver;                // admitted-gradient counter (the model version), server control buffer
  unsigned long long* batch_ctr;  // FCFS microbatch counter
  float* shard[kP2PMaxRanks];   // shard k's base (element i at shard[i >> shard_shift][i & (2^shift - 1)])
  int shard_shift, nshards;
  int excl;                     // 1: this rank is the only writer (world 1): plain read-modify-write
  float* w;                     // local fp32 master [n] (pull destination)
  const float* g;               // local fp32 gradient [n]
  long long n;
  unsigned* vpulled;            // local: vp of the last admission (the applied count its weights contained)
  unsigned* applied;            // shared: gradients whose every add has landed (ps_device.h; null: legacy)
  unsigned* audit;              // optional local [audit_cap][3] (version at admission, vp, decision) rows
  long long audit_cap;
  unsigned long long* stats;    // local [8]: accepted, rejected, sum staleness, max staleness, CAS retries, err,
                                //            no-op steps after the schedule finished
  unsigned* herr;               // host-mapped mirror of the error bits (host watchdog, no HIP call)
  unsigned* scratch;            // local [64 + kPSMaxGrid] protocol words (async_ps.hip; kPSVMin starts at ~0)
  const long long* perm;        // [nbatches][B] example ids (nullptr: no index staging)
  long long* idx;               // [B] staged ids of the claimed microbatch
  long long* bid_out;           // local: claimed microbatch (epoch << 32 | batch), -1 = dataset finished
  // epoch-scoped completion accounting (shared, nullptr = legacy unbounded counter): sched[0] dataset
  // epoch, sched[1] batches completed in it; sched_ctr[0..3] completed, redispatched, skipped,
  // duplicate; done_epoch[b] = e + 1 once batch b is applied in epoch e; claimed_epoch[b] likewise
  // for its first dispatch
  unsigned* sched;
  unsigned long long* sched_ctr;
  unsigned* done_epoch;
  unsigned* claimed_epoch;
  const float* lr_dev;          // device learning rate (the store's hyper[0]); null: use lr
  long long nbatches, timeout_ticks;
  int B, max_stale, max_epochs;  // max_epochs 0 = unbounded
  float lr;
  // owner-applies (owner_ring > 0; csrc/async_ps.hip): no per-element remote atomics.  An admitted gradient
  // of sequence number q is written (plain system-scope stores) into ring slot q % owner_ring of every
  // shard's inbox, then flagged there; a pull that takes a shard's drain lock adds its flagged slots into
  // the shard in sequence order and publishes how many are drained (pref[k]).  "Fully applied" = min pref.
  float* inbox[kP2PMaxRanks];   // owner k's inbox: owner_ring slots of its shard length, then owner_ring flags
  unsigned* pref;               // shared [nshards] drained-sequence counts
  unsigned* dlock;              // shared [nshards] drain locks (0 free, rank + 1 held): any pulling rank drains
  int owner_ring, rank;
};
constexpr int kPSMaxGrid = 64;

// Device FedSGD count barrier on the parameter server's shards (csrc/fedsgd_ps.hip): the reference
// FederatedServer's version gate and K-upload barrier, K < W allowed (late uploads are dropped).
constexpr int kFedMaxK = 32;  // the landed / bad slot masks are 32-bit
struct FedArgs {
  unsigned* seq;                 // control: version seqlock (2v: version v stable; odd: being applied)
  unsigned long long* tick;      // control: (seq << 32) | tickets taken for that version
  unsigned long long* land;      // control: (seq << 32) | mask of the slots whose gradient has landed
  unsigned long long* bad;       // control: (seq << 32) | mask of the slots landed as bad (torn or lost)
  float* shard[kP2PMaxRanks];    // master shards (element i: shard[i >> shift][i & mask])
  float* slot[kP2PMaxRanks];     // per rank: K slot shards (slot t of element i: slot[i >> shift][t << shift | i & mask])
  int shard_shift, nshards, K;
  long long n;
  float* w;                      // local master (pull destination)
  const float* g;                // local gradient (upload)
  unsigned* scratch;             // local protocol words (fedsgd_ps.hip)
  unsigned long long* stats;     // local [8]: admitted, stale, full, failed, versions applied, versions recovered,
                                 //            -, error bits
  unsigned* audit;               // optional local rows [audit_cap][3]: (seqlock word pulled, decision, slot)
  long long audit_cap;
  const float* lr_dev;           // device learning rate (null: lr)
  float lr;
  long long timeout_ticks;
  unsigned* herr;
  int drop_land;                 // fault injection (tests): take the ticket, then store and land nothing
};
hipError_t fed_pull(const FedArgs& a, hipStream_t st);
hipError_t fed_upload(const FedArgs& a, hipStream_t st);
hipError_t fed_apply(const FedArgs& a, hipStream_t st);
constexpr int kPSVMinWord = 4;  // scratch word of the refresh minimum (ps_device.h kPSVMin)
constexpr int kPSDecisionWord = 3;  // scratch word of the tagged admission decision (ps_device.h kPSDecision)
constexpr long long kPSMaxBatches = 1 << 20;  // capacity of the shared completion arrays
hipError_t ps_fetch_pull(const PSArgs& a, hipStream_t st);
// apply-path calibration: mode 0 per-element CAS adds of 0, mode 1 owner-applies stores / loads (async_ps.hip)
hipError_t ps_calibrate(const PSArgs& a, int mode, hipStream_t st);
hipError_t ps_apply(const PSArgs& a, hipStream_t st);
// exclusive writer (one rank): admission of this step's gradient, the next microbatch's claim and index
// staging, in one workgroup; the update itself is the optimizer launch gated on the decision
hipError_t ps_excl_step(const PSArgs& a, hipStream_t st);
// shard self-test: every rank adds (rank + 1) * (j + 1) to word j of every shard's test area, n words
hipError_t ps_selftest_add(const PSArgs& a, float* const* words, int n, float rank1, hipStream_t st);


// Whole-network LeNet-5 training step (csrc/lenet_fused.hip): conv5x5x6 'same' + pool, conv5x5x16 +
// pool, dense 400-120-84-10, softmax-CE, full backward.  Conv weights are read from the fp32 master,
// dense weights from the bf16 compute copies ([Npad16][Kpad32] and the dgrad layout).
constexpr int kLeNetPW1 = 0, kLeNetPB1 = 150, kLeNetPW2 = 156, kLeNetPB2 = 2556, kLeNetConvParams = 2572;
constexpr int kLeNetConvStride = 2576;  // floats per workgroup row of the conv partial buffer
struct LeNetArgs {
  const unsigned char* x_u8;  // [nrows][784] uint8 dataset read through idx (or null)
  const bf16* x_bf;           // [B][784] bf16 batch (when x_u8 is null)
  const long long* idx;       // [B] dataset rows (or null: row r of the batch)
  long long nrows;
  float scale;                // uint8 -> value scale
  const int* labels;          // read through idx like the images
  const float *w1, *b1, *w2, *b2;  // fp32 master: conv1 [6][25], [6]; conv2 [16][150], [16]
  const bf16 *d1w, *d1wt, *d2w, *d2wt, *d3w, *d3wt;  // [128][416] [400][128] [96][128] [128][96] [16][96] [96][32]
  const float *d1b, *d2b, *d3b;
  float* conv_part;           // [nblocks][kLeNetConvStride] per-workgroup conv gradient partials
  float* loss_part;           // [nblocks][2]
  bf16 *h0T, *h1T, *h2T;      // [400|120|84][ldt] transposed dense inputs
  bf16 *dz1T, *dz2T, *dz3T;   // [120|84|10][ldt] transposed dense output gradients
  float* logits;              // [B][10] (nullable)
  int prep;                   // 1: launch the fragment prep kernel first (0: the optimizer rebuilt them)
  const void* frag;           // [37][64] x 8 bf16 conv weight fragments of this step (written by the prep launch)
  const unsigned char* ftab;  // [98][2][16] conv2 dgrad gather table (lenet_tables)
  const unsigned short* pxtab;  // [800] conv2 output row -> pool1 pixel (lenet_tables)
  unsigned long long* stamps; // diagnostic phase clocks [grid][16] (lenet_set_stamps), or null
  int B, ldt;
  float grad_scale;
  // async PS: one extra workgroup (index nblk) admits this step's gradient while the others train, so the
  // reduce launch's owners find the decision already published (csrc/lenet_fused.hip)
  int nblk, ps_admit;
  // ps_admit with one rank (the exclusive writer, lenet_reduce_kernel<3>): the admission also advances the
  // launch epoch and publishes the applied count itself (the reduce launch has no arrival protocol)
  int ps_excl;
  // images per train workgroup (lenet_ipw): 8, or fewer at small batches -- more workgroups, each running
  // only its images' share of the per-image phases (the critical path of a small step is one workgroup's)
  int ipw;
  PSArgs ps;
};
struct LeNetDense {
  const bf16* dzT;
  const bf16* hT;
  float* gw;  // [N][K]
  float* gb;  // [N]
  int N, K, tiles;
};
// Fused update of the LeNet-5 step: the reduce kernel applies the SGD update to every parameter it
// finalises (no optimizer launch), stages the next batch's indices and scatters every updated conv
// weight into the next step's MFMA fragments (lenet_frag_scatter).
struct LeNetSgd {
  float* master;
  float* mom;          // null without momentum
  bf16* wbf;
  const float* hyper;  // [lr, momentum, wd, grad_scale, nesterov]
  ParamDesc d[10];     // w1, b1, w2, b2, dense (w, b) x 3 (ParamStore order)
  const long long* src;  // index stream [nsteps][B] (null = off), cursor, dst
  long long* cursor;
  long long* dst;
  int B, nsteps;
  float* run_stats;    // nullable: [loss sum, correct, updates] accumulated by the loss workgroup
  void* frag;          // fragment buffer of the next step
};
// Contiguous copy of what the reduce launch indexes at run time (filled by lenet_train from the fields
// below): the kernel stages it into LDS with one parallel vector load from the kernel-argument segment.
struct LeNetRedTab {
  LeNetDense L[3];
  float* g[10];    // gradient output per descriptor: w1, b1, w2, b2, dense (w, b) x 3
  ParamDesc d[10];
};
struct LeNetRedArgs {
  LeNetRedTab tab;
  const float* conv_part;  // [nblk][kLeNetConvStride]
  const float* loss_part;
  float* stats;  // [2] loss sum, correct
  float *g_w1, *g_b1, *g_w2, *g_b2;
  LeNetDense L[3];
  int nblk, ldt, nconv_slots, dense_tiles;  // dense_tiles: 32 x 32 units (L[l].tiles per layer)
  int kcols;       // batch columns summed (round32(B)); ldt is the row stride of H^T / dZ^T
  int chunk_cols;  // batch columns per dense job (a multiple of 32; chunk c = XCD c's train workgroups)
  float* slabs;      // [slots][8 chunks][1024] job partials (write-through), chunk 0 then the owner's sum
  unsigned* tickets;  // [slots] arrival tickets, zero between launches (the last arriver resets)
  // optional snapshot [2][2550] of the conv kernels' weights (w1, w2) and momentum (m1, m2; null = 0)
  const float *w1, *w2, *m1, *m2;
  float* snap;
  int sgd_on;
  LeNetSgd sgd;
  // world > 1 (requires sgd_on): the owner of every slot sums its values over the ranks through the
  // in-kernel LL exchange (LL slot = slot) before applying the update, so a multi-rank step is still two
  // launches
  int ll_on;
  LLComm ll;
  // job workgroups G (0 = one per job); fewer when ranks time-share one GPU (each then runs several jobs
  // and owns up to 16 slots), so that every rank's waiting workgroups fit on the chip at once
  int exch_blocks;
  // asynchronous SGD against the device parameter server (requires sgd_on for the compute-copy layout):
  // the gradient is admitted by the lock-free version CAS (staleness bound ps.max_stale) and added to the
  // SHARDED master (w <- w - lr * g), the local master / bf16 copies / conv fragments are refreshed from
  // the values the adds produced (or, for a rejected gradient, the current ones), and the next microbatch
  // is claimed and staged: an async step is train + this launch (csrc/lenet_fused.hip, csrc/ps_device.h)
  int ps_on;
  PSArgs ps;
  unsigned long long* stamps;  // diagnostic: [grid][16] wall-clock marks per phase (scripts/lenetstamps.py), or null
  // successor ownership (succ = 1; one job per workgroup): job (slot s, chunk c) publishes its partial as
  // 8-byte {launch epoch, value} granules; the workgroups of slot s + 1 (plus one owner-only group after the
  // last slot) each own one eighth of slot s's positions and sum its 8 chunks in chunk order (no ticket,
  // no slab reload: one hand-off).  A workgroup waits only on lower-indexed ones.
  int succ;
  unsigned long long* gran;  // [slots][8 chunks][1024]
  unsigned* gran_ep;         // [grid] per-workgroup launch counters (each workgroup reads / bumps its own)
  unsigned* gran_err;        // sticky: a granule wait timed out
  unsigned* slot_arr;        // [slots] async PS: owners of a slot done (the eighth arrives for the slot)
  // async PS with one rank (mode 3: the synchronous owners' update gated on the train launch's admission):
  // every new weight is also written here (the rank's master shard); null otherwise
  float* mirror;
  // small batches, one rank, sync (set by lenet_train): one workgroup per slot reduces it over the whole
  // batch and applies its update itself (no 8-way split, no hand-off)
  int solo;
};
// The reference CNN's conv block (csrc/kcnn_fused.hip): conv1 3x3x1->32 + ReLU, conv2 3x3x32->32 + ReLU,
// 2x2 max-pool [+ folded dropout], input 28x28x1, in one forward and one backward launch (+ reduce).
struct KcnnArgs {
  const uint8_t* x_u8;  // uint8 dataset [nrows][784] (read through idx), or
  const bf16* x_bf;     // bf16 rows [.][784] (through idx with scale, or the batch itself)
  const long long* idx;
  long long nrows;
  float scale;
  const bf16* w1;   // conv1 compute copy [32][kpad1] (k = tap)
  const float* b1;  // [32]
  const bf16* w2;   // conv2 compute copy [32][288] (k = tap * 32 + ci)
  const bf16* w2t;  // conv2 dgrad copy [32 ci][288] (tap * 32 + n)
  const float* b2;
  bf16* pooled;     // [B][144][32]
  uint8_t* code;    // [B][144][32] argmax position 0..3, 4 = no gradient
  const bf16* dyp;  // [B][144][32] gradient of the pooled (post-dropout) map
  float* slab2;     // [blocks][32][289]
  float* slab1;     // [blocks][32][10]
  int B, kpad1;
  DropSpec drop;
  unsigned long long* stamps;  // profiling aid (kcnn_set_stamps): backward [G][2 images][16] phase clocks, or null
};
void kcnn_set_stamps(void* buf);
int kcnn_blocks(int B);
size_t kcnn_slab_floats(int B);
hipError_t kcnn_fwd(const KcnnArgs& a, hipStream_t st);
hipError_t kcnn_bwd(const KcnnArgs& a, float* g_w1, float* g_b1, float* g_w2, float* g_b2, long long* step_inc,
                    hipStream_t st);
// The reference CNN's dense head (csrc/khead.hip): dense 4608 -> 128 ReLU [+ folded dropout] -> dense C
// softmax-CE, forward, loss and both data gradients in ONE launch (split-K over 8 workgroups per 32 rows).
constexpr int kKHeadRows = 32, kKHeadChunks = 8, kKHeadN1 = 128;
struct KHeadArgs {
  const bf16* p;      // [B][K] dense1 input
  bf16* pT;           // [K][ldt] its transpose (dense1 weight-gradient operand)
  bf16* dp;           // [B][K] dense1 data gradient (nullable)
  const bf16* w1;     // [128][ldw1] forward layout
  const bf16* w1t;    // [>= K][128] data-gradient layout
  const float* b1;    // [128] (nullable)
  const bf16* w2;     // [16][128]
  const bf16* w2t;    // [128][32]
  const float* b2;    // [C] (nullable)
  DropSpec drop;      // dropout after dense1 (folded into its epilogue)
  float dh_scale;     // dense2's dX scale (the folded dropout's 1/(1-p); 1 = none)
  float dp_scale;     // dense1's dX scale (a dropout folded below dense1; 1 = none)
  int dp_mask;        // relu'(P) on dense1's dX
  bf16 *h1T, *dz1T, *dz2T;  // [128][ldt], [128][ldt], [C][ldt]
  float* logits;      // [B][C] fp32 (nullable)
  const int* labels;  // labels (through idx when idx != null)
  const long long* idx;
  long long nrows;
  float grad_scale;
  float* loss_part;   // [cdiv(B, 16)][2] (the fused head kernels' layout)
  float* slab;        // [ntiles][8][32 * 128] split-K partials
  bf16* dz1;          // [ntiles][32][128] published dZ1 tiles
  unsigned* sync;     // [ntiles] tickets, [ntiles] flags, {launch tag, finished workgroups}
  unsigned long long* stamps;  // profiling aid (khead_set_stamps): [G][16] phase clocks, or null
  int B, K, C, ldt, ldw1, ntiles, G;
};
void khead_set_stamps(void* buf);
void khead_set_grid_cap(int cus);
// Weight gradients of that head (csrc/khead.hip khead_wgrad_kernel): dW = dZ^T X over the whole batch
// in 64 x 32 output tiles (bias = the column k == K of ones), plus the loss partials -> stats.
struct KHeadWgradLayer {
  const bf16* a;  // dZ^T [N][ldt]
  const bf16* b;  // X^T [K][ldt]
  float *gw, *gb;  // [N][K], [N] (nullable)
  int N, K, nblk, kblk;
};
struct KHeadWgradArgs {
  KHeadWgradLayer L[2];
  int ldt, jobs, nloss;
  const float* loss_part;
  float* stats;
};
hipError_t khead_wgrad(KHeadWgradArgs a, hipStream_t st);
size_t khead_ws_floats(int B, int K);
size_t khead_lds(int K);
bool khead_supported(int K, int C);
hipError_t khead_train(KHeadArgs a, hipStream_t st);
int lenet_dense_part_floats(int B);  // reduce scratch: job slabs, arrival tickets, granules, launch counters
void lenet_red_bind_scratch(float* dense_part, LeNetRedArgs& r);  // points r's scratch fields into it
int lenet_red_err_offset();  // float offset of the granule error word in that scratch
size_t lenet_train_lds();
int lenet_blocks(int B);
hipError_t lenet_train(const LeNetArgs& a, LeNetRedArgs r, hipStream_t st);
void lenet_set_stamps(void* buf);
size_t lenet_frag_bytes();

// Classifier evaluation metrics (csrc/metrics.hip): out = [sum of the per-example loss, correct].
enum MetricKind {
  kMetricMSE = 0, kMetricAbs = 1, kMetricHinge = 2, kMetricHuber = 3, kMetricLog = 4, kMetricSigmoidCE = 5,
  kMetricSoftmaxCE = 6, kMetricCategoricalCE = 7
};
hipError_t classifier_metrics(const float* z, const int* labels, int B, int C, int kind, int softmax, float* out,
                              hipStream_t st);

// Generic Keras layers (csrc/act.hip): standalone activations, sigmoid-CE loss, general pooling.
enum ActKind {
  kActLinear = 0, kActRelu = 1, kActRelu6 = 2, kActSigmoid = 3, kActTanh = 4, kActElu = 5, kActSelu = 6,
  kActSoftplus = 7, kActSoftsign = 8, kActHardSigmoid = 9, kActSwish = 10, kActExp = 11
};
hipError_t act_fwd(const bf16* x, bf16* y, long long n, int kind, hipStream_t st);
hipError_t act_bwd(const bf16* x, const bf16* dy, bf16* dx, long long n, int kind, int in_relu, hipStream_t st);
hipError_t sigmoid_ce(const float* logits, const int* labels, bf16* dlogits, float* stats, int B, int C, int ldl,
                      int ldg, float grad_scale, hipStream_t st);
struct Pool2DGeom {
  int B, H, W, C, OH, OW;
  int ph, pw, sh, sw, pt, pl;  // window, stride, top / left padding
};
hipError_t pool2d_fwd(const bf16* x, bf16* y, const Pool2DGeom& g, int avg, hipStream_t st);
hipError_t pool2d_bwd(const bf16* x, const bf16* dy, bf16* dx, const Pool2DGeom& g, int avg, int in_relu,
                      hipStream_t st);

// Direct convolution for C_in <= 4 (csrc/smallc.hip); igemm_fwd / igemm_wgrad dispatch to it.
bool smallc_fwd_supported(const IGemmArgs& a, int mode);
hipError_t smallc_fwd(const IGemmArgs& a, hipStream_t st);
bool smallc_wgrad_supported(const WgradArgs& a, int mode);
hipError_t smallc_wgrad(const WgradArgs& a, float* ws, size_t ws_floats, hipStream_t st);

}  // namespace dfa
