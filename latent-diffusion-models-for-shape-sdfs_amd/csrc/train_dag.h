// The persistent training-step kernel's job table (host builder: denoiser_train.hip
// build_dag; device: train_dag.hip).  Internal, not part of the ABI.
//
// One DDPM training step (config 2: q_sample -> denoiser forward -> eps-MSE -> backward ->
// AdamW) is a DAG of NODES: the 15 grouped-GEMM problems of the launch-per-GEMM step
// (denoiser_train.hip forward / backward, recorded, not re-derived), the input preparation, the
// bias-gradient / loss sums (each fused with its bias's AdamW update) and the AdamW tiles of
// every weight.  A node is a set of JOBS (kBand x kBand output tiles, kBand-row x 64-column
// input chunks, groups of 64 x 64 parameter tiles); a job waits on counters its producers raise:
//   * band dependency: the producer's kBand-row band counter of the consumer's own band reaches
//     the producer's tiles per band (a layer of the residual chain needs only its band of the
//     layer below -- no grid-wide barrier between dependent GEMMs);
//   * all dependency: the producer's all-jobs counter reaches its job count (weight gradients
//     contract over the whole batch; AdamW waits for its gradient and for the last reader of
//     the weight copy it rewrites).
// Jobs are dealt to 8 queues (workgroup w pulls from queue w % 8, so under the round-robin
// dispatch one queue's workgroups share an XCD and its L2: speed only).  Every queue lists its
// jobs in the global node order, which is topological, so with every workgroup resident the
// earliest unfinished job always has its inputs: no deadlock.
#pragma once
#include "ldm_internal.h"

namespace ldm {
namespace dag {

constexpr int kQueues = 8;
constexpr int kBand = 64;               // rows of a band (= a row node's GEMM tile rows)
constexpr int kThreads = 512;           // the kernel's workgroup: 8 waves, one per CU
// GEMM job configurations (train_dag.hip TileCfg): tile rows x cols
enum TileKind : int { TILE_K2 = 0 /* 64 x 64, two k-groups */, TILE_ROW = 1 /* 64 x 128 */,
                      TILE_W = 2 /* 128 x 128 */,
                      TILE_K2L = 3 /* 64 x 64, two k-groups, 128-deep stages (kgp 2) */ };
inline int tile_rows(int kind) { return kind == TILE_W ? 128 : 64; }
inline int tile_cols(int kind) { return kind == TILE_K2 || kind == TILE_K2L ? 64 : 128; }
constexpr int kMaxDeps = 4;
constexpr int kMaxNodes = 96;
constexpr int kAdamGroup = 4;           // AdamW 64 x 64 tiles per job (one acquire for 4)
constexpr int kCtrStride = 32;          // counters 128 bytes apart (one line each)
// sync region (unsigned words, each on its own 128-byte line): queue heads, the claim lists'
// heads, exit counter, status, then the counters
constexpr int kSyncHead = 0;                    // kQueues lines
constexpr int kSyncHead2 = kQueues;             // 2 kQueues lines (the claim scheduler's lists)
constexpr int kSyncExit = 3 * kQueues;          // 1 line
constexpr int kSyncStatus = 3 * kQueues + 1;
constexpr int kSyncCtr0 = 3 * kQueues + 2;      // first counter line

enum NodeType : int { N_GEMM = 0, N_PREP = 1, N_SUM = 2, N_ADAM = 3 };

struct Node {
    int type;
    int tiles_m, tiles_n, nk;       // GEMM: tile x tile grid, k-steps (64 deep); PREP: tiles_m
                                    // row bands x tiles_n 64-column chunks of [xt | e]; SUM:
                                    // 1 x 1; ADAM: tiles_m 64-row tiles x tiles_n jobs of
                                    // kAdamGroup of the node's nk 64-column tiles
    int ndep;
    int dep_ctr[kMaxDeps];          // counter index (band dependency: + the consumer's band)
    int dep_band[kMaxDeps];
    unsigned dep_target[kMaxDeps];
    int out_band;                   // first of tiles_m band counters (-1: none)
    int out_all;                    // the all-jobs counter
    int signal;                     // 1: a later node waits on this node's counters (release +
                                    // count after every job); 0: nobody does, the job just ends
    int pin_eps;                    // GEMM: P_in is the launch's eps (the LOSS target)
    int tile;                       // GEMM: TileKind
    int row;                        // GEMM / PREP: rows are the batch's (64-row band counters)
    int kgp;                        // GEMM: 0, or the k-group period of the launch path's tile
                                    // (two accumulators alternating every kgp 64-deep k-steps)
    int stat;                       // GEMM: bit 0 / 1: every segment's A / B is a weight copy
                                    // no job writes before the step's last read of it -- may be
                                    // loaded through the L2 (plain) instead of sc1 (kDbgWeightsL2)
    int adam;                       // SUM / ADAM: tensor index (-1: no update)
    int amode;                      // ADAM: adamw_tile mode (0 all; 1 p, m, v; 2 bf16 copies)
    int col_off;                    // ADAM: first 64-column tile of this node in the tensor
    // SUM: dst[c] = scale * sum_{r < rows} src[r ld + c], c < len; dst NULL: the launch's
    // loss_out
    const float* src;
    float* dst;
    int rows, len, ld;
    float scale;
    // PREP (prep_inputs_kernel<true>'s arithmetic)
    const float* sab;
    const float* s1mab;
    const float* emb;
    int B, Bp, D, TE;
    unsigned short *xt_b, *xt_T, *e_b, *e_T;
    ldm_gemm_prob_t P;              // GEMM (KB 64, LDS-transposed epilogue)
};

struct Table {
    uint64_t hash;                  // of the inputs the table was built from (launch checks it)
    int n_nodes, n_counters, n_entries, n_tensors, grid;
    int qlen[kQueues], qoff[kQueues];   // queue q: entries[qoff[q] .. qoff[q] + qlen[q])
    // the claim scheduler's lists (kDbgClaim): per queue q the chain jobs (row nodes, prep) at
    // [q] and the others at [q + kQueues], each in node order
    int qlen2[2 * kQueues], qoff2[2 * kQueues];
    ldm_adamw_tensor_t tensor[LDM_ADAMW_MAX_TENSORS];
    Node node[kMaxNodes];
    // uint32 entries[n_entries] follow: node << 16 | job
};

constexpr int kMaxEntries = 16384;
constexpr unsigned kDbgFences = 128;
constexpr unsigned kDbgClaim = 256;     // claim scheduler: take only READY jobs, chain first
constexpr unsigned kDbgWeightsL2 = 512; // weight operands through the L2 (Node::stat; measured
                                        // ~1 % slower than sc1 at config 2, profiles/r05v)
inline size_t table_bytes() { return sizeof(Table) + sizeof(uint32_t) * kMaxEntries; }
inline size_t sync_bytes(int n_counters) {
    return (size_t)(kSyncCtr0 + n_counters) * kCtrStride * sizeof(unsigned);
}
constexpr int kMaxCounters = 512;

// Per-launch arguments (the inputs that change every step).
struct LaunchArgs {
    const Table* tab;       // device copy (read-only during the launch)
    unsigned* sync;         // zero before the first launch; every launch leaves it zeroed
                            // except the status word
    uint64_t hash;
    const float* x0;
    const float* eps;
    const int32_t* t;
    float* loss_out;
    const float* d_hyper;   // device AdamW scalars (graph replays) or NULL: hy below
    float hy[7];
    unsigned spin_limit;    // microseconds a dependency wait may take before it gives up
    unsigned dbg;           // diagnostics (ldm_dev_train_dag_flags): bit t skips the compute of
                            // node type t (jobs still wait and signal); kDbgFences: add the
                            // agent release / acquire fences to every hand-off (A/B);
                            // kDbgClaim: the claim scheduler (train_dag.hip)
};

// device side (train_dag.hip)
int dag_launch(const LaunchArgs& a, int grid, hipStream_t s);
int dag_grid(int* grid);    // resident workgroups of the kernel on this device, a multiple of 8

}  // namespace dag
}  // namespace ldm
