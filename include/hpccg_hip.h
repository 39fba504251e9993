/*
 * hpccg_hip.h -- C ABI of the MI355X-native HPCCG hot path (libhpccg_hip.so).
 *
 * Plain pointers and sizes only. Every entry point replaces one interface of
 * the reference (Dart120/HPCCG-SYCL, file:line cited per function). Return
 * value: 0 on success, a negative HPCCG_HIP_E* code on failure (the message
 * is available from hpccg_hip_last_error()). The reference itself has no
 * error path (HPCCG.cpp:401 always returns 0; fatal conditions abort).
 *
 * Layout on the device (per GPU / rank):
 *   matrix   SELL-512-A where it applies (every slice has at most 32 distinct
 *            column - row offsets and every row's columns ascend: stencils):
 *            slices of 512 consecutive rows, slot j of a slice holds every
 *            row's entry at the slice's j-th smallest offset (0.0 where the row
 *            has none), fp64, 8 B per slot, offsets per slice. Otherwise
 *            SELL-512: slot-major vals[slice][slot][512] fp64 + cols int32
 *            (padding col = -1). Entry order per row is the caller's order in
 *            both, so every row sum rounds like the reference. DESIGN.md 3.
 *   vectors  fp64, length padded to a multiple of 512; p carries the halo:
 *            [ghost_lo | local rows | ghost_hi] (z-slab plan) or
 *            [local rows | externals] (gather plan).
 */
#ifndef HPCCG_HIP_H
#define HPCCG_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

struct HPC_Sparse_Matrix_STRUCT;
typedef struct hpccg_hip_matrix hpccg_hip_matrix; /* opaque, device resident */

#define HPCCG_HIP_OK 0
#define HPCCG_HIP_EINVAL (-1)  /* bad argument / shape */
#define HPCCG_HIP_EHIP (-2)    /* HIP runtime error */
#define HPCCG_HIP_ERCCL (-3)   /* RCCL error */
#define HPCCG_HIP_ENOMEM (-4)  /* device allocation failed */
#define HPCCG_HIP_EPLAN (-5)   /* no halo plan for this partition (e.g. halo mode 1 and a
                                  matrix coupling ranks other than r-1, r+1) */
#define HPCCG_HIP_ENODEV (-6)  /* no HIP device */

/* ---- library ---------------------------------------------------------- */
int hpccg_hip_abi_version(void);            /* == 2 */
const char* hpccg_hip_last_error(void);     /* thread-local message */
int hpccg_hip_device_count(int* count);
int hpccg_hip_set_device(int device);       /* one GPU per rank/process */

/* ---- communicator: replaces MPI_COMM_WORLD in ddot.cpp:75-85,
 *      exchange_externals.cpp:51-131 and make_local_matrix.cpp:185-201.
 *      RCCL over xGMI; one rank per GPU. Without a communicator the
 *      library runs single-GPU (nranks = 1). ---------------------------- */
int hpccg_hip_comm_unique_id(unsigned char id_out[128]);
int hpccg_hip_comm_init(const unsigned char id[128], int nranks, int rank);
/* Host-bootstrapped communicator (replaces MPI_Init / MPI_COMM_WORLD's setup
 * role, main.cpp:131-132 and make_local_matrix.cpp:185-201; no RCCL): the
 * ranks' setup exchanges (the halo plan's all-gather, the IPC handles of the
 * peer mailboxes and of r, the self-tests' verdicts) go through the caller's
 * all-gather -- allgather(send, recv, bytes, ctx) must place every rank's
 * `bytes` bytes into recv in rank order and return 0 -- e.g. gloo from
 * torch.distributed. The CG iteration then makes no collective call at all:
 * the two scalars are summed inside the kernels through IPC-mapped mailboxes
 * (ddot.cpp:75-85) and each rank pulls its z-slab ghost planes of r from its
 * neighbours' memory (exchange_externals.cpp:51-131). Several ranks may share
 * one GPU (RCCL refuses that). Matrix creation is collective and fails on
 * every rank (HPCCG_HIP_EPLAN) when that transport is not available: the
 * gather halo plan, a matrix without a SELL-512-A image, or a self-test that
 * failed on any rank. The kernel-level sparsemv and ddot exchange through the
 * callback. hpccg_hip_comm_destroy ends it. */
typedef int (*hpccg_hip_allgather_fn)(const void* send, void* recv, unsigned long long bytes, void* ctx);
int hpccg_hip_comm_init_host(int nranks, int rank, hpccg_hip_allgather_fn allgather, void* ctx);
int hpccg_hip_comm_destroy(void);
int hpccg_hip_comm_size(int* nranks, int* rank);
/* The communicator in use: 0 none (one rank), 1 RCCL, 2 host-bootstrapped. */
int hpccg_hip_comm_mode(int* mode);
/* Host-value all-reduce over the communicator (main.cpp:206-208,
 * compute_residual.cpp:73): op 0 = sum, 1 = min, 2 = max. In place. */
int hpccg_hip_comm_allreduce_host(double* vals, int n, int op);
/* The job's in-kernel transport verdicts (collective over the communicator;
 * matrix creation calls it after the self-tests): local = this rank's own
 * results {peer all-reduce, halo pull, production protocol}, verdict = the
 * job's, the same on every rank -- the peer all-reduce and the pull stay on
 * only where every rank passed, the protocol counts only where both did, and
 * a protocol failure on any rank turns both off everywhere (RCCL carries the
 * scalars and r's planes; a host-bootstrapped job refuses the matrix).
 * Replaces nothing in the reference (its exchange has one transport). Debug:
 * HPCCG_DBG_FAIL_PROTO in a rank's environment makes its protocol self-test
 * report a failure, to exercise the collective fallback. */
int hpccg_hip_transport_verdict(const int local[3], int verdict[3]);
/* Device name and compute-unit count of the current device. */
int hpccg_hip_device_name(char* buf, int cap, int* compute_units);
/* Runtime identity of this process (diagnostics; replaces nothing in the
 * reference, whose MPI path is compiled out: main.cpp:131-132):
 * ints_out = {ranks of the RCCL communicator as RCCL counts them
 * (ncclCommCount; 0 without one), this rank (ncclCommUserRank), ncclGetVersion,
 * hipRuntimeGetVersion, hipDriverGetVersion, current device}; the device's PCI
 * bus id; the shared objects the library's RCCL and HIP entry points resolved
 * to (dladdr). Buffers may be NULL. */
int hpccg_hip_runtime_info(int ints_out[6], char* pci_bus_id, int pci_cap, char* rccl_path, char* hip_path,
                           int path_cap);

/* ---- host-side input (the reference's generate_matrix.cpp:196-307) ------
 * Builds the reference HPC_Sparse_Matrix for rank `rank` of `size`
 * z-stacked slabs (global column indices), plus x0 = 0, b, xexact = 1.
 * use_7pt selects the 7-point stencil (generate_matrix.cpp:219). Arrays are
 * allocated with new[]; free with hpccg_free_problem. */
int hpccg_generate_matrix(int nx, int ny, int nz, int rank, int size, int use_7pt,
                          struct HPC_Sparse_Matrix_STRUCT** A, double** x, double** b,
                          double** xexact);
/* read_HPC_row (read_HPC_row.cpp:217-373, Mode 2 input): the rows of rank
 * `rank` of `size` (the reference's block partition, remainder spread over the
 * first ranks) of the system in data_file, global columns; x (initial guess),
 * b and xexact from the file. Free with hpccg_free_problem. Returns
 * HPCCG_HIP_EINVAL with a message on a missing or malformed file (the
 * reference prints "Error: Cannot open file" and exits). Host only. */
int hpccg_read_HPC_row(const char* data_file, int rank, int size, struct HPC_Sparse_Matrix_STRUCT** A,
                       double** x, double** b, double** xexact);
void hpccg_free_problem(struct HPC_Sparse_Matrix_STRUCT* A, double* x, double* b,
                        double* xexact);

/* ---- device matrix -------------------------------------------------------
 * hpccg_hip_matrix_create: converts the caller's HPC_Sparse_Matrix
 * (HPC_Sparse_Matrix.hpp:54-85; read-only, caller keeps ownership, global
 * column indices) to SELL-512 (+ -L, -C where they apply) and uploads it.
 * The halo plan replaces make_local_matrix.cpp:58-610: the z-slab plan when
 * every rank's external columns are contiguous planes of rank+-1, else the
 * gather plan (see hpccg_hip_set_halo_mode). Collective over the
 * communicator when nranks > 1. */
int hpccg_hip_matrix_create(const struct HPC_Sparse_Matrix_STRUCT* A, hpccg_hip_matrix** out);
/* Same from plain CSR (row_ptr[nrow+1] int64, cols int32 global, vals fp64). */
int hpccg_hip_matrix_create_csr(int nrow, int start_row, int total_nrow, const long long* row_ptr,
                                const int* cols, const double* vals, hpccg_hip_matrix** out);
/* Generate the stencil matrix directly on the GPU in SELL-512 layout
 * (same entries, same order as generate_matrix.cpp:251-289), with b and
 * xexact on the device. Rank/size from the communicator. */
int hpccg_hip_matrix_generate(int nx, int ny, int nz, int use_7pt, hpccg_hip_matrix** out);
int hpccg_hip_matrix_destroy(hpccg_hip_matrix* M);
/* Halo plan for matrices created after this call (process-wide): 0 auto (the
 * z-slab plan when it serves every rank -- contiguous ghost planes from rank+-1
 * only -- else the gather plan), 1 slab only (HPCCG_HIP_EPLAN otherwise), 2
 * gather always. The gather plan is make_local_matrix.cpp:58-610: external
 * columns numbered after the local rows, grouped by owning rank in the
 * reference's order, send lists learned from the owners' requests, and each
 * halo exchange packs p at the requested rows (exchange_externals.cpp:51-131).
 * The device generator always builds slab plans. */
int hpccg_hip_set_halo_mode(int mode);
/* Matrices created afterwards keep their SELL-512 image beside SELL-512-A
 * (process-wide; default 0 frees it once the A image exists). Only for
 * kernel A/B comparisons ("spmv_kernel" 0 on a stencil matrix). */
int hpccg_hip_set_keep_sell(int keep);
/* Placement probe of matrices created afterwards (process-wide): 0 off (the
 * default), -1 auto (6 candidates when the SELL-512-A values exceed 512 MB,
 * off otherwise and for in-process group members), 1..16 candidates. See
 * hpccg_hip_probe_placement. Replaces nothing in the reference. */
int hpccg_hip_set_placement_probe(int tries);
/* nrow, ncol (incl. ghosts), stored nnz, matrix slots (incl. padding),
 * ghost_lo, ghost_hi, SpMV kernel, uniform slot count (0 = per slice). */
int hpccg_hip_matrix_info(const hpccg_hip_matrix* M, long long info_out[8]);
/* Device pointers owned by M: b, x0 (zeros) and xexact of a generated matrix. */
int hpccg_hip_matrix_vectors(hpccg_hip_matrix* M, double** b_dev, double** x0_dev,
                             double** xexact_dev);

/* ---- solver: replaces HPCCG() HPCCG.cpp:312-402 ----------------------------
 * Host-pointer form (b, x host; x in/out). times[0..6]:
 * [0] solve total, [1] DDOT (incl. all-reduce), [2] WAXPBY, [3] SPARSEMV,
 * [4] all-reduce, [5] halo exchange, [6] setup (H2D of b, x).
 * Residual lines (HPCCG.cpp:356,372-373) are printed by rank 0 when
 * print != 0. */
int hpccg_hip_solve(hpccg_hip_matrix* M, const double* b, double* x, int max_iter,
                    double tolerance, int* niters, double* normr, double* times, int print);
/* Device-pointer form: b_dev, x_dev already in HBM (x_dev in/out); nothing
 * crosses PCIe inside. The bench's timed step. */
int hpccg_hip_solve_device(hpccg_hip_matrix* M, const double* b_dev, double* x_dev, int max_iter,
                           double tolerance, int* niters, double* normr, double* times,
                           int print);
/* normr computed in each iteration of the last solve: out[0] = initial
 * residual, out[k] = iteration k (k <= niters). Returns entries written. */
int hpccg_hip_last_trace(const hpccg_hip_matrix* M, double* out, int cap);
/* Solver options (set / get). Twelve settings of the solve:
 *   "spmv_kernel"   -1 auto (default), 0 SELL-512 gather, 1 SELL-512-A with x
 *                   read at the slice's offsets, 2 SELL-512-A with x from LDS
 *                   windows shared by slice pairs; get: the kernel in use
 *   "use_graph"     replay CG iterations from hipGraphs (default 1; every rank
 *                   count, RCCL calls captured; falls back to eager launches if
 *                   the capture is refused); get "graph_used": the last solve did
 *   "graph_chunk"   iterations per graph (default 32). Rounded up to an even
 *                   count with the fused update (each captured launch bakes in
 *                   the parity of its k) and to a multiple of the p ring when a
 *                   halo is exchanged; get returns the effective count
 *   "fuse_p"        -1 auto / 0 off: p = r + beta p formed inside the SpMV
 *                   (pair and direct kernels; on several ranks with the z-slab
 *                   plan, through the r-halo exchange; get "rhalo": in use)
 *   "fold"          dots completed inside the producing kernel through
 *                   self-validating slots: -1 / 1 both (default), 0 neither
 *                   (a k_finalize launch per dot)
 *   "fuse_update"   -1 auto (on) / 0 / 1: one rank, direct kernel: the update
 *                   runs as trailing blocks of the SpMV launch (one launch per
 *                   iteration; same bits); 2: also in an in-process group with
 *                   the peer all-reduce (tests: small members only)
 *   "resident_update" -1 auto (default): the persistent launch (k_cg_persist,
 *                   one launch per solve) where every pair block of the matrix
 *                   fits on the chip at once, else the per-iteration resident
 *                   pair launch (k_spmv_ar) where that fits; 1 k_spmv_ar only;
 *                   0 off. get: 8 persistent, 1 k_spmv_ar, 0 neither. A
 *                   resident solve whose wait expired is re-run with the other
 *                   launch; get "resident_retries" counts such re-runs
 *   "x_defer"       x += alpha p deferred over the p ring: 1 = every x_ring-th
 *                   update applies it to all rows; 2 (default) = trailing blocks
 *                   of every SpMV launch apply it to the 1/(x_ring-1) of the
 *                   slices whose turn it is (SELL-512-A kernels; reads back 1
 *                   with the others); 0 = every iteration (same bits all ways)
 *   "x_ring"        p ring length = x deferral depth, 2..64; -1 auto: 32 for
 *                   matrix images over 512 MB, else 8
 *   "a2_ring"       pair kernel: value slots in flight per wave through its
 *                   LDS-DMA ring, -1 auto (3), 0 register loads (uniform widths
 *                   27 and 7; other depths measured slower and are refused)
 *   "peer_allreduce" -1 auto (default: an RCCL job whose creation-time
 *                   self-test passed on every rank, and the force_comm 2
 *                   emulation), 0 RCCL, 1 on: the two CG scalars summed inside
 *                   the kernels through IPC-mapped mailboxes
 *   "halo_pull"     r-halo by pull: -1 auto (default), 0 off (the RCCL plane
 *                   group / peer copies), 1 k_pull before each SpMV launch,
 *                   2 in-launch: the iteration's last launch pulls once its
 *                   r.r completion is in (needs the peer all-reduce; auto picks
 *                   it there, else 1); 3 diagnostics (force_comm 2 only):
 *                   in-launch with no rows
 * Diagnostics:
 *   "event_timing" 1 = eager launches with hipEvents around every SpMV and
 *                   update (hpccg_hip_kernel_times)
 *   "spin_budget_us" bound of every in-kernel wait (the dot slots, the fused
 *                   update's p.Ap total), default 1000000. A wait that outlives
 *                   it records itself on the device and ends the solve: the
 *                   call returns HPCCG_HIP_EHIP naming the wait (block, group,
 *                   iteration, dot), every rank of an RCCL job returns it, and
 *                   the dot slots are reset before the next solve
 *   "force_comm"    1-rank communicator: 1 = route the two CG scalars through
 *                   ncclAllReduce; 2 = also the multi-rank iteration (a
 *                   plane-sized ncclSend/ncclRecv to itself as the halo);
 *                   captured in the graph like N > 1
 *   "dbg_timeline"  1 = the ring pair kernel (width 27, ring 3) records a
 *                   per-block timeline (hpccg_hip_diag_timeline)
 *   "dbg_withhold"  (guard test) slice + 1 whose p.Ap partial is never
 *                   published, so the solve must time out (0 = off)
 *   "dbg_resident_stall" (retry test) 1 = the resident launches' p.Ap wait
 *                   never sees the total, so it expires
 * get only: "has_sell", "has_a", "has_pairs", "a_width", "lds_doubles", "nt",
 * "nt_store", "halo_mode", "num_external", "group_fold" (the last in-process
 * group solve summed its dots in its members' kernels), "resident_retries",
 * "peer_auto_ok", "pull_auto_ok", "proto_auto_ok", "persist_auto_ok" (the
 * creation-time self-tests' verdicts), "placement_pick", "device_bytes" (device memory M
 * holds). None of the options changes a computed value: every kernel, fusion
 * and fold setting gives the same bits. Variants that measured even or slower
 * than these defaults were removed. */
int hpccg_hip_set_option(hpccg_hip_matrix* M, const char* key, long long value);
int hpccg_hip_get_option(const hpccg_hip_matrix* M, const char* key, long long* value);
/* hipEvent kernel timings of the last solve with event_timing on:
 * out[0] SpMV total ms, out[1] SpMV launches, out[2] fused-update total ms,
 * out[3] update launches (launches that did work, i.e. <= niters + 1). */
int hpccg_hip_kernel_times(const hpccg_hip_matrix* M, double out[4]);
/* The same per iteration (0 = the prologue): out[2i] SpMV ms, out[2i + 1]
 * update ms, up to cap iterations; returns the count (diagnostics). */
int hpccg_hip_kernel_times_iter(const hpccg_hip_matrix* M, double* out, int cap);
/* Diagnostic: average duration (hipEvents, solver stream) of `reps`
 * back-to-back launches of SpMV kernel `kernel` (prologue form) on the
 * resident p; kernel 9 streams the SELL-512-A values alone (8 B x slots read,
 * 8 B x n written: the rocprofv3 FETCH_SIZE calibration). */
int hpccg_hip_diag_spmv(hpccg_hip_matrix* M, int kernel, int reps, double* avg_us);
/* Diagnostic: move one device buffer to a new allocation (contents copied;
 * the old one is held until the matrix is destroyed, so the new one lands on
 * other physical memory): which & 255 = 0 the SELL-512-A values, 1 the p
 * ring, 2 r, 3 Ap, 4 x; which >> 8 = the allocation: 0 hipMalloc, 1
 * physically contiguous (hipDeviceMallocContiguous -- corrupts other buffers
 * of the process on this stack, DESIGN.md 5: diagnostics only), 5 fine-grained
 * (hipDeviceMallocFinegrained), 6 uncached, 2/3/4 the VMM API
 * (hipMemCreate + hipMemMap) at 2 MB / 64 MB / 1 GB virtual alignment. The
 * new virtual address goes to *va_out (may be NULL). For measuring the effect
 * of physical placement on the kernels' rate. Replaces nothing in the
 * reference. */
int hpccg_hip_diag_realloc(hpccg_hip_matrix* M, int which, unsigned long long* va_out);
/* The CG iteration rate of a large matrix depends on the physical HBM
 * placement of its values and p ring (306-350 us per 200^3 SpMV on one box).
 * Times a few eager CG iterations (median SpMV + update, scratch b and x; a
 * rank of an RCCL job is timed alone, no collective call) on the current
 * placement, then on up to `tries` candidate allocations of the values
 * (plain hipMalloc: contiguous ones corrupted other buffers; copied) and
 * keeps the fastest, then likewise of the p ring, r and
 * Ap (zeroed); frees the rest. A phase stops early, keeping its best so far,
 * when free memory falls below the candidate size + 8 GiB. Results are
 * unchanged (bitwise). Option "placement_pick" reads the kept candidates: one
 * byte per buffer, values | ring << 8 | r << 16 | Ap << 24 (0 = the placement
 * before the probe). */
int hpccg_hip_probe_placement(hpccg_hip_matrix* M, int tries);
/* The last probe's times (us per iteration: [0] the placement before the
 * probe, then the values, ring, r and Ap candidates in turn): returns their
 * count, copies up to cap. */
int hpccg_hip_diag_placement(const hpccg_hip_matrix* M, double* us_out, int cap);
/* Diagnostic (option dbg_timeline 1): block timeline of the last SpMV launch
 * that ran an iteration, 8 words per row, s_memrealtime stamps (100 MHz).
 * Ring pair kernel (width 27, ring 3), one row per pair: block | HW_ID << 32,
 * entry, iteration state read, windows staged, slot loop done, epilogue done,
 * XCC id, iteration k. Direct kernel with the fused update (the 100^3 and 7-pt
 * defaults), one row per block of the launch: block | HW_ID << 32, entry,
 * state read (unit block) or p.Ap ready (update block), slot loop done, end,
 * role (0 unit, 1 side flush, 2 ghost store, 3 update), XCC id, 0. Up to cap
 * rows (cap x 8 words); returns the row count. Replaces nothing in the
 * reference (its TICK/TOCK classes are per kernel). */
int hpccg_hip_diag_timeline(const hpccg_hip_matrix* M, unsigned long long* out, int cap);
/* Debug (canary mode: HPCCG_CANARY=1 in the environment when the library
 * first allocates): every matrix buffer is allocated with a 64 KB canary of
 * a NaN pattern no kernel stores before and after it, and every solve checks
 * every canary of the process when it ends (HPCCG_HIP_EHIP naming the buffer
 * and the byte range on a trip). This checks them now (device-wide sync
 * first): returns the number of tripped canaries and describes up to 8 in
 * report; *enabled = whether canary mode is on. Replaces nothing in the
 * reference (its solver touches only its own work vectors, HPCCG.cpp:327-329). */
int hpccg_hip_diag_canary_check(int* enabled, char* report, int cap);
/* Diagnostic (host only, no GPU): the folded dot completion's plan for a
 * launch of `units` units (spu = 1 slice or 2 slices each) on `grid` blocks
 * dealt over the 8 XCDs (rev: the update's reversed order): for each group of
 * 64 slices the unit whose block waits for the group (the group's largest
 * block index), and the top group. Returns the group count. Replaces nothing
 * in the reference (ddot.cpp:60-88 sums on one thread). */
int hpccg_hip_diag_slot_plan(int units, int grid, int spu, int rev, int* last_unit, int cap, int* top_group);

/* ---- in-process rank group --------------------------------------------------
 * The z-slab decomposition of one process's RCCL job (make_local_matrix.cpp
 * :58-610 + exchange_externals.cpp:51-131 + the MPI_Allreduce in ddot.cpp),
 * driven from ONE host thread: member r is rank r of nranks (devices[r], or
 * the current device for all when devices is NULL; several ranks may share a
 * device). Halo planes move by peer copies between the members' streams and
 * the two CG scalars are summed in rank order by one lane on rank 0's
 * device. The kernels are the multi-rank ones an RCCL job runs; only the
 * transport differs. nranks <= 16. Not inside an RCCL job (nranks > 1 there). */
int hpccg_hip_group_generate(int nx, int ny, int nz, int use_7pt, int nranks, const int* devices,
                             hpccg_hip_matrix** out);
/* Member r from CSR rows [start_row[r], start_row[r] + nrow[r]) of the global
 * matrix (global columns, z-slab halo only; HPCCG_HIP_EPLAN otherwise). */
int hpccg_hip_group_create_csr(int nranks, const int* devices, const int* nrow, const int* start_row,
                               int total_nrow, const long long* const* row_ptr, const int* const* cols,
                               const double* const* vals, hpccg_hip_matrix** out);
/* HPCCG() over the group: b_dev[r], x_dev[r] are rank r's local rows on its
 * device (x in/out). niters, normr and times (rank 0's stamps) as
 * hpccg_hip_solve_device; every member's hpccg_hip_last_trace is set. */
int hpccg_hip_group_solve(hpccg_hip_matrix* const* Ms, int nranks, const double* const* b_dev,
                          double* const* x_dev, int max_iter, double tolerance, int* niters, double* normr,
                          double* times);

/* ---- kernel level, device pointers, synchronous ----------------------------
 * hpccg_hip_sparsemv: HPC_sparsemv.cpp:68-89. x_dev has the local rows (the
 * halo is exchanged from it on multi-rank runs), y_dev local rows. */
int hpccg_hip_sparsemv(hpccg_hip_matrix* M, const double* x_dev, double* y_dev);
/* ddot.cpp:60-88: deterministic two-stage reduction; all-reduced over the
 * communicator when nranks > 1. Result to host. */
int hpccg_hip_ddot(int n, const double* x_dev, const double* y_dev, double* result);
/* waxpby.cpp:69-93: w = alpha*x + beta*y (w may alias x or y). */
int hpccg_hip_waxpby(int n, double alpha, const double* x_dev, double beta, const double* y_dev,
                     double* w_dev);

/* ---- drop-in driver: HPCCG.hpp:61-63 with C linkage. Prepares the device
 * matrix (cached per A: keyed by the address AND a fingerprint of the sizes,
 * row lengths, column indices and values, so a matrix re-created at the same
 * address or edited in place is converted again), then runs hpccg_hip_solve.
 * On a cached image the solve starts at once and the fingerprint is taken
 * beside it; x and the residual lines are written only once it matched (else
 * the image is rebuilt and the solve re-run from the caller's x).
 * A localised matrix (local_ncol > local_nrow) is refused (HPCCG_HIP_EPLAN). */
int hpccg_hip_HPCCG(struct HPC_Sparse_Matrix_STRUCT* A, double* b, double* x, int max_iter,
                    double tolerance, int* niters, double* normr, double* times);
/* Frees the cached device matrix of A (destroyMatrix of this package calls
 * it); returns 1 if there was one. */
int hpccg_hip_dropin_release(const struct HPC_Sparse_Matrix_STRUCT* A);
/* 1 if a device matrix is cached for A. */
int hpccg_hip_dropin_cached(const struct HPC_Sparse_Matrix_STRUCT* A);

/* ---- host-only helpers (no GPU needed; used by the CPU test suite) -------
 * Converts CSR rows [0, nrow) with global columns into the SELL-512 image the
 * device uses. First call with vals/cols = NULL to size: returns the number
 * of SELL slots; slice_base has nslices+1 entries (units of 512 slots). */
long long hpccg_sell_build(int nrow, long long col_base, long long ncol_ext, const long long* row_ptr,
                           const int* cols, const double* vals, unsigned int* slice_base,
                           int* sell_cols, double* sell_vals);
/* z-slab halo plan for a CSR slab: ghost_lo/ghost_hi from the column range
 * (see hpccg_hip_matrix_create). Returns 0 or HPCCG_HIP_EPLAN. */
int hpccg_halo_plan(int nrow, int start_row, int total_nrow, const long long* row_ptr,
                    const int* cols, int plan_out[4]);
/* What rank `rank` sends (make_local_matrix.cpp:286-587 handshake, z-slabs):
 * info has 4 ints per rank {nrow, ghost_lo, ghost_hi, start_row} (the
 * all-gather the library does at matrix creation); sends[0] = rows to
 * rank-1 (its first rows), sends[1] = rows to rank+1 (its last rows). */
int hpccg_slab_plan(int nranks, int rank, const int* info, int sends[2]);
/* The local half of the gather plan (make_local_matrix.cpp:96-200) for one
 * rank's rows (global columns): the external columns in local-index order
 * (ext_global[j] is local column nrow + j: grouped by owning rank, groups in
 * order of first appearance, first appearance inside a group) and the receive
 * runs per owner. info as for hpccg_slab_plan. Arrays of at least cap
 * entries, filled when large enough; counts always. Host only. */
int hpccg_gather_plan(int nranks, const int* info, int nrow, int start_row, const long long* row_ptr,
                      const int* cols, int cap, int* ext_global, int* num_external, int* nrecv, int* recv_rank,
                      int* recv_off, int* recv_cnt);

#ifdef __cplusplus
}
#endif
#endif
