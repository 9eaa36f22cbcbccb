/*
 * dlrm_hip.h — C ABI of the MI355X (gfx950) DLRM embedding + feature-interaction hot path.
 *
 * This is the drop-in boundary for darchr/DLRM.jl.  Every entry point replaces one operator
 * of the reference's hot path (citations are /root/reference paths):
 *
 *   dlrm_maplookup        EmbeddingTables.maplookup(PreallocationStrategy(P), tables, sparse)
 *                         called at src/model/model.jl:161; semantics pinned by
 *                         test/model/embedding_update.jl:23-33, test/model/interact.jl:168-171,
 *                         test/integration.jl:10-11 (the package itself is un-vendored).
 *   dlrm_interact_fwd     (dot::DotInteraction)(x, ys)           src/model/interact.jl:394-411
 *                         = fast_vcat (:271-281) + process_batches (:449-467)
 *                           + process_slice! (:338-362) + triangular_slice_kernel! (:64-75)
 *   dlrm_interact_bwd     dot_back / process_batches_back        src/model/interact.jl:415-489
 *                         (fused unpack :154-173, gemmavx! :318-326, sumavx :329-336)
 *   dlrm_indexer_*        EmbeddingTables.SparseIndexer()        src/train/train.jl:276-281
 *   dlrm_triangular_slice(_back), dlrm_self_batched_mul(_back)
 *                         Implementation 2 of the interaction (dot_interaction, the default of
 *                         dlrm(), model.jl:180): src/model/interact.jl:176-215, :503-551
 *   dlrm_sgd_update       EmbeddingTables.update!(Descent(lr), tables, grads, indexers;
 *                         num_splits, nthreads)                  src/train/train.jl:283-290
 *                         (grads = maplookup pullback = SparseEmbeddingUpdate views of dt,
 *                         test/train/backprop.jl:147-158, src/validation.jl:125-146)
 *
 * Conventions
 *  - All tensors are caller-owned DEVICE memory (from dlrm_malloc, hipMalloc or torch).
 *    Nothing on a launch path allocates or synchronises, so every launching call can be
 *    captured into a hipGraph.
 *  - Layout: a Julia column-major (D, N) matrix is C row-major [N][D].  The lookup output
 *    (P + D*T) x B is C [B][out_ld] with table t at columns out_offset + t*D; the interaction
 *    output (d + F(F-1)/2 + padding) x B is C [B][out_ld].
 *  - Indices are int32 or int64, laid out [T][batch*lookups] with a per-table stride
 *    (sample-major within a table: position p = b*lookups + k, as load_inputs reshapes them,
 *    src/data/criteo.jl:551-557).  index_base is 1 for Julia / DACLoader indices, 0 for
 *    PyTorch / HDF5 indices.
 *  - Errors: every function returns a dlrm_status (0 = OK, negative = error) and no C++
 *    exception crosses the ABI.  dlrm_last_error(ctx) describes the last failure.
 *    Out-of-range indices never fault: kernels skip them and raise a device-side flag that
 *    dlrm_check_bounds() turns into DLRM_E_INDEX (the reference throws BoundsError).
 *  - Threading: one ctx = one device + one stream; calls are asynchronous on that stream;
 *    a ctx must not be used from two host threads at once.
 */
#ifndef DLRM_HIP_H
#define DLRM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLRM_HIP_ABI_VERSION 1

typedef enum {
    DLRM_OK = 0,
    DLRM_E_ARG = -1,         /* invalid argument (shape, null pointer, dtype)          */
    DLRM_E_HIP = -2,         /* HIP runtime error                                       */
    DLRM_E_INDEX = -3,       /* an index was outside [index_base, index_base + nrows)   */
    DLRM_E_UNSUPPORTED = -4, /* valid request this build does not implement             */
    DLRM_E_NOMEM = -5,       /* device allocation failed                                */
    DLRM_E_STATE = -6        /* object used in the wrong state (e.g. indexer not built) */
} dlrm_status;

typedef enum { DLRM_F32 = 0, DLRM_BF16 = 1 } dlrm_dtype;
typedef enum { DLRM_I32 = 0, DLRM_I64 = 1 } dlrm_itype;

/* dlrm_sgd_update flags */
#define DLRM_UPDATE_ATOMIC 1u   /* float atomics straight into the rows: fastest to launch,
                                   NOT bitwise reproducible (fp32 tables only)            */
#define DLRM_UPDATE_PREBUILT 2u /* the indexer was already built from these indices by
                                   dlrm_indexer_build (e.g. on a side stream during the
                                   forward pass); skip rebuilding it                     */

typedef struct dlrm_ctx dlrm_ctx;         /* device + stream + error word                  */
typedef struct dlrm_tables dlrm_tables;   /* Vector{SimpleEmbedding{Static{D}}} on device  */
typedef struct dlrm_indexer dlrm_indexer; /* Vector{SparseIndexer}: per-table dedupe state */

/* ---- context ---------------------------------------------------------------------- */
int dlrm_abi_version(void);
int dlrm_ctx_create(int device, void* stream /* hipStream_t, NULL = default */, dlrm_ctx** out);
int dlrm_ctx_destroy(dlrm_ctx* ctx);
int dlrm_ctx_set_stream(dlrm_ctx* ctx, void* stream);
const char* dlrm_last_error(const dlrm_ctx* ctx);
/* Diagnostics: on = 1 installs handlers that print a native backtrace to stderr on SIGSEGV, SIGBUS
 * or SIGABRT and then run the previous handler (0 restores them).  Not for production use. */
int dlrm_debug_fatal_trace(int on);
int dlrm_sync(dlrm_ctx* ctx);
/* Synchronises, reads and clears the device out-of-range flag raised by any kernel since
 * the previous call.  DLRM_E_INDEX if it was set. */
int dlrm_check_bounds(dlrm_ctx* ctx);
/* Bounds errors without a per-step synchronisation (the deferred update! of the drop-in chain).
 * The step backward (dlrm_step_bwd / _prepare, backward launch) copies the flag into host memory
 * owned by the ctx as it reads it (one thread's store); for other sequences
 * dlrm_error_snapshot queues a copy of the device flag into host memory owned by the ctx (on the
 * ctx stream; capturable, no synchronisation); dlrm_error_peek reads the last copy that has landed
 * (no GPU call; 0 = no error seen yet).  A kernel that finds the device flag set writes no table
 * row, so the tables keep the state before the failing step until dlrm_check_bounds reports and
 * clears the flag (it also clears the host copy). */
int dlrm_error_snapshot(dlrm_ctx* ctx);
int dlrm_error_peek(const dlrm_ctx* ctx, unsigned* word);

/* ---- device memory (so a host language without ROCm bindings can own buffers) ------- */
int dlrm_malloc(dlrm_ctx* ctx, size_t bytes, void** dptr);
int dlrm_free(dlrm_ctx* ctx, void* dptr);
int dlrm_memcpy_h2d(dlrm_ctx* ctx, void* dst, const void* src, size_t bytes); /* synchronous */
int dlrm_memcpy_d2h(dlrm_ctx* ctx, void* dst, const void* src, size_t bytes); /* synchronous */
/* Page-locks a host range for direct DMA (hipHostRegister) / releases it; dlrm_memcpy_h2d_async
 * queues a copy on the ctx stream and returns (the source must stay unchanged until the stream
 * reaches it; from registered memory the copy is a DMA with no staging). */
int dlrm_host_register(void* ptr, size_t bytes);
int dlrm_host_unregister(void* ptr);
int dlrm_memcpy_h2d_async(dlrm_ctx* ctx, void* dst, const void* src, size_t bytes);

/* ---- embedding tables --------------------------------------------------------------- */
/* Registers T tables of one dtype and feature size `dim` (SimpleEmbedding{Static{dim}}).
 * data[t] points at a device [nrows[t]][dim] row-major table.  The table memory stays
 * caller-owned; dlrm_sgd_update mutates it in place. */
int dlrm_tables_create(dlrm_ctx* ctx, int num_tables, int dim, int dtype,
                       void* const* data, const int64_t* nrows, dlrm_tables** out);
int dlrm_tables_destroy(dlrm_tables* tables);

/* maplookup(PreallocationStrategy(out_offset), tables, sparse):
 *   out[b][out_offset + t*dim + c] = sum_{k<lookups} table_t[idx_t[b*lookups + k] - base][c]
 * Columns [0, out_offset) are not touched (they are reserved for x, interact.jl:264-270).
 * lookups = 1 is the one-hot copy (bit-exact); lookups > 1 sums in k order in fp32. */
int dlrm_maplookup(dlrm_ctx* ctx, const dlrm_tables* tables,
                   const void* indices, int itype, int64_t table_stride, int index_base,
                   int batch, int lookups,
                   void* out, int64_t out_ld, int64_t out_offset);

/* dlrm_maplookup with a general output row map (the table-sharded exchange layout,
 * dlrm.jl_amd/sharded.py: every peer's block written in place, no repack):
 *   row b of table t -> out + (b / block_rows) * block_stride + (b % block_rows) * out_ld
 *                           + out_offset + t * table_stride        (elements)
 * dlrm_maplookup(...) == dlrm_maplookup_blocked(..., table_stride = dim, block_rows = batch,
 * block_stride = 0).  No reference counterpart (DLRM.jl is single-process). */
int dlrm_maplookup_blocked(dlrm_ctx* ctx, const dlrm_tables* tables,
                           const void* indices, int itype, int64_t table_stride, int index_base,
                           int batch, int lookups, void* out, int64_t out_ld, int64_t out_offset,
                           int64_t out_table_stride, int64_t block_rows, int64_t block_stride);

/* Row scatter of the exchange (sharded backward: dt's table columns -> per-owner blocks):
 *   dst + dst_base[t] + b * dst_ld[t]  <-  src + b * src_ld + src_offset + t * dim
 * for b < batch, t < num_tables, dim elements of esize (2 or 4) bytes; dst_base / dst_ld are
 * device arrays of num_tables int64 (elements).  No reference counterpart. */
int dlrm_scatter_rows(dlrm_ctx* ctx, int esize, int num_tables, int batch, int dim,
                      const void* src, int64_t src_ld, int64_t src_offset, void* dst,
                      const int64_t* dst_base, const int64_t* dst_ld);

/* ---- pairwise dot interaction -------------------------------------------------------- */
/* (dot::DotInteraction)(x, ys): copies x[b][0:d] into ys[b][0:d] (fast_vcat), views
 * ys[b][0:F*d] as T_b = [F][d], and writes
 *   out[b] = [ x_b | Z[i][j] for i = 1..F-1, j = 0..i-1 | 0 * padding ],  Z = T_b T_b^T
 * dtype applies to x, ys and out (bf16 in, fp32 accumulate, bf16 out). */
int dlrm_interact_fwd(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch,
                      const void* x, int64_t x_ld, void* ys, int64_t ys_ld,
                      void* out, int64_t out_ld, int padding);

/* maplookup(PreallocationStrategy(d), tables, sparse) followed by (dot::DotInteraction)(x, ys)
 * as ONE launch (model.jl:161-163 with the bottom MLP already applied): every gathered row is
 * loaded once into MFMA fragments and written to ys from registers, so ys is never re-read.
 * ys and out receive exactly what dlrm_maplookup(out_offset = d) + dlrm_interact_fwd write
 * (bit-identical); shapes without a fused kernel fall back to those two launches.
 * ys may be NULL when the caller will not read the lookup output (a training step whose
 * backward is dlrm_interact_bwd_gather): then only out is written, and shapes without a
 * fused kernel return DLRM_E_UNSUPPORTED.  Requires tables->dim == d; dtype is the tables'. */
int dlrm_lookup_interact_fwd(dlrm_ctx* ctx, const dlrm_tables* tables,
                             const void* indices, int itype, int64_t table_stride, int index_base,
                             int batch, int lookups,
                             const void* x, int64_t x_ld, void* ys, int64_t ys_ld,
                             void* out, int64_t out_ld, int padding);

/* ---- Implementation 2 of the interaction, as separate operators --------------------------
 * dot_interaction (src/model/interact.jl:503-517; the default of dlrm(), model.jl:180) composes
 * fast_vcat + self_batched_mul + triangular_slice; dlrm_interact_fwd / dlrm_interact_bwd are that
 * composition and its pullback in one launch each.  These are the pieces and their rrules, for
 * callers that compose them as the reference does.  Layouts: Z, dZ (sz, sz, B) = [B][sz][sz]
 * (batch stride given, element [b][col][row] = Julia z[row, col, b]); the slice (ncols, B) = [B][ld];
 * T (d, F, B) = [B][F][d] (batch stride t_ld).
 * dlrm_triangular_slice       triangular_slice (:176-191): out[b][col(col-1)/2 + row] = z[b][col][row],
 *                             row < col (triangular_slice_kernel! order, :64-75).  Bit-exact copy.
 * dlrm_triangular_slice_back  its rrule (:193-215): a[b][col][row] = dy[b][col(col-1)/2 + row] for
 *                             row < col, 0 elsewhere (triangular_slice_back_kernel!, :104-120);
 *                             symmetric != 0: also the lower triangle (the fused add-transpose form,
 *                             :150-171).  Bit-exact.
 * dlrm_self_batched_mul       self_batched_mul (:526-537): z[b] = T_b^T T_b (full, F x F), fp32
 *                             accumulation, stored in dtype.  F <= 90.
 * dlrm_self_batched_mul_back  its rrule (:539-551): dt[b] = T_b (dz_b + dz_b^T), fp32 out.  F <= 90. */
int dlrm_triangular_slice(dlrm_ctx* ctx, int dtype, int sz, int batch, const void* z, int64_t z_batch_stride,
                          void* out, int64_t out_ld);
int dlrm_triangular_slice_back(dlrm_ctx* ctx, int dtype, int sz, int batch, const void* dy, int64_t dy_ld, void* a,
                               int64_t a_batch_stride, int symmetric);
int dlrm_self_batched_mul(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch, const void* t, int64_t t_ld,
                          void* z, int64_t z_batch_stride);
int dlrm_self_batched_mul_back(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch, const void* t,
                               int64_t t_ld, const void* dz, int64_t dz_batch_stride, float* dt, int64_t dt_ld);

/* dot_back(dot, dout, t, d, padding): S_b = symmetric zero-diagonal unpack of
 * dout[b][d : d + F(F-1)/2];  dt[b] = S_b T_b  ([F][d], fp32, x-rows included as the
 * reference returns them);  dx[b] = dout[b][0:d] + dt[b][0:d]  (fp32).
 * t is the ys buffer of the forward pass (dtype as dout). */
int dlrm_interact_bwd(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch,
                      const void* dout, int64_t dout_ld, int padding,
                      const void* t, int64_t t_ld,
                      float* dx, int64_t dx_ld, float* dt, int64_t dt_ld);

/* dot_back as dlrm_interact_bwd, with T_b rebuilt from x (row 0) and the tables' rows of the
 * sample's one-hot indices (rows 1..F-1) instead of read from a materialized ys: the same
 * values while the tables are unchanged since the forward (recomputation, not a cache).
 * lookups must be 1; dtype is the tables' (dout and x in it); dx, dt fp32 as above.
 * indexer (may be NULL): also builds it from the same indices, as dlrm_indexer_build would --
 * in the same launch where the shape allows (its workgroups sort while the backward's stream),
 * so the step's dlrm_sgd_update can pass DLRM_UPDATE_PREBUILT.
 * Declared after the indexer type below; see the SparseIndexer section. */

/* ---- sparse indexer + SGD scatter update --------------------------------------------- */
int dlrm_indexer_create(dlrm_ctx* ctx, int num_tables, int64_t max_lookups_per_table,
                        dlrm_indexer** out);
int dlrm_indexer_destroy(dlrm_indexer* indexer);
/* Dedupe: per table, group the lookup positions by row -> one segment per distinct row
 * holding the positions that hit it in ascending order (segment order is unspecified).
 * Asynchronous; device-side counts only.  By batch * lookups positions per table: <= 4096 in LDS
 * (one workgroup per table), <= 8192 in LDS over 4 parts, <= 32768 the bag build (count, place by
 * part, per-part sort: pooled bags, round 6; DLRM_BAG_WAVE=0 selects the next form instead), above
 * that the hash build.  Out-of-range indices are left out and raise the bounds flag. */
int dlrm_indexer_build(dlrm_ctx* ctx, dlrm_indexer* indexer, const dlrm_tables* tables,
                       const void* indices, int itype, int64_t table_stride, int index_base,
                       int batch, int lookups);
/* The split form of the indexer that dlrm_step_bwd consumes (one-hot batches): positions whose
 * row is hit once are flagged (dlrm_step_bwd updates those rows inside the backward), the other
 * rows are listed for the apply.  dlrm_step_fwd builds it inside the forward's launch; building
 * it here instead lets a caller prepare the NEXT batch's indexer ahead of time (it depends only
 * on the indices, e.g. on a side stream during the current step) and run a step as
 * dlrm_lookup_interact_fwd(ys = NULL) + dlrm_step_bwd. */
int dlrm_indexer_build_split(dlrm_ctx* ctx, dlrm_indexer* indexer, const dlrm_tables* tables,
                             const void* indices, int itype, int64_t table_stride, int index_base,
                             int batch);
/* Inspection (synchronous): unique-row count of one table; if rows != NULL copies up to
 * cap unique rows (0-based, in segment order); if positions != NULL copies up to cap
 * positions (b*lookups + k) grouped by segment and the segment starts (cap+1 entries). */
int dlrm_indexer_read(dlrm_ctx* ctx, const dlrm_indexer* indexer, int table,
                      int64_t* num_unique, int64_t* rows, int64_t* positions,
                      int64_t* seg_start, int64_t cap);

/* The training step's split build of `indices` on the ctx's stream -- a side stream: it depends on
 * the indices only -- so that the dlrm_step_fwd of the same indices only gathers (the build
 * dlrm_step_bwd_prepare runs inside an apply launch, as its own launch).  One-hot, batch <= 32768
 * positions per table (16 table parts per 2048 positions, one wave each; above 2048 positions the
 * scan build: 8 or 16 waves per workgroup scan the table, int32 indices with 16-B aligned tables and
 * batch % 4 == 0, else the build in rounds), any number of tables (tables x capacity < 2^31); the
 * indexer must have been created for >= batch positions.  Replaces the SparseIndexer() build of
 * train.jl:276-281 ahead of the step (also the table-sharded update's build over the global
 * batch).  Out-of-range indices are left out of the build and raise the ctx's bounds flag through
 * the lookup / forward of the same indices, or the apply of this indexer (dlrm_sgd_update PREBUILT,
 * dlrm_step_bwd) -- not from the build itself, which may run beside a step that reads the flag to
 * decide its writes.  DLRM_E_UNSUPPORTED: a shape the wave build does not take (use
 * dlrm_indexer_build). */
int dlrm_indexer_prepare(dlrm_ctx* ctx, dlrm_indexer* indexer, const dlrm_tables* tables,
                         const void* indices, int itype, int64_t table_stride, int index_base, int batch);

/* Device bytes the indexer holds, all allocated by dlrm_indexer_create: the per-part arrays (~92 B
 * per position slot; the wave builds pack a table's parts back to back, so any of them fits cap
 * slots per table -- x 8 for a cap of 4097..8192, the in-LDS parts build's layout), the wave
 * build's flat item lists (<= 256 B per slot) and HBM sort scratch (20 B, cap > 2048), and above
 * 4096 the hash arrays.  Nothing grows on a later build (26 tables x 16384: ~0.2 GB). */
int dlrm_indexer_bytes(const dlrm_indexer* indexer, int64_t* bytes);
/* Kept for callers of round 5's layout, which re-carved the indexer on its first wave build of
 * > 2048 positions: the packed layout needs no re-carving, so this only validates batch. */
int dlrm_indexer_reserve(dlrm_ctx* ctx, dlrm_indexer* indexer, int batch);
/* The wave build's chunk limit for this indexer's later builds (16 or 32, default 32): segments of
 * at most this many positions become chunk items (one lane group each), longer ones hot-slice items
 * (a workgroup each).  16 turns the 17..32-position segments of uniform one-hot batches (the
 * 105-row Kaggle table) into one-round items (DESIGN.md §3 "Round 6").  Deterministic either way; a
 * 17..32-position segment is summed in a different (fixed) order, so its fp32 rounding may differ. */
int dlrm_indexer_set_chunk(dlrm_ctx* ctx, dlrm_indexer* indexer, int max_positions);
/* Parts per table of this indexer's later wave builds of <= 2048 positions per table (the step's
 * in-apply / forward-launch builds, dlrm_indexer_prepare): 16 (the default, 0), 32 or 64; one wave
 * sorts each part.  More parts shorten the build's chain and add workgroups beside the apply: a
 * win where the apply's items are light (rows <= 256 B: D = 16 fp32, Terabyte bf16 rows), a loss
 * at 512-B rows (DESIGN.md §3 "Round 6").  Results are identical for any setting. */
int dlrm_indexer_set_parts(dlrm_ctx* ctx, dlrm_indexer* indexer, int parts);

/* Host-side state of the last build (no GPU call): a mask of DLRM_IX_* bits.  SINGLES_DONE: a
 * split backward (dlrm_step_bwd) has stepped this build's once-hit rows, so its dt holds only
 * the repeated rows' gradients.  (The Julia shim's pullback state, DLRMHip.jl `st.bwd`.) */
enum { DLRM_IX_BUILT = 1, DLRM_IX_SPLIT = 2, DLRM_IX_PREPARED = 4, DLRM_IX_SINGLES_DONE = 8 };
int dlrm_indexer_state(const dlrm_indexer* indexer, unsigned* state);

/* Backward of a training step without a materialized ys (see above). */
int dlrm_interact_bwd_gather(dlrm_ctx* ctx, const dlrm_tables* tables, dlrm_indexer* indexer,
                             const void* indices, int itype, int64_t table_stride, int index_base,
                             int batch, int lookups, const void* x, int64_t x_ld,
                             const void* dout, int64_t dout_ld, int padding,
                             float* dx, int64_t dx_ld, float* dt, int64_t dt_ld);

/* dlrm_interact_bwd_gather for the table-sharded backward: dx as there, and table t's dt row of
 * sample b written straight to dst + dst_base[t] + b * dst_ld[t] (fp32; dst_base / dst_ld device
 * arrays of num_tables int64 elements, the send layout of dlrm_alltoall_bwd), i.e. the backward
 * and dlrm_scatter_rows in one launch; dt's x rows are not written.  Needs 16-B aligned rows, x,
 * dx and dst (DLRM_E_UNSUPPORTED otherwise).  No reference counterpart. */
int dlrm_interact_bwd_blocked(dlrm_ctx* ctx, const dlrm_tables* tables,
                              const void* indices, int itype, int64_t table_stride, int index_base,
                              int batch, const void* x, int64_t x_ld, const void* dout, int64_t dout_ld,
                              int padding, float* dx, int64_t dx_ld, float* dst,
                              const int64_t* dst_base, const int64_t* dst_ld);

/* update!(Descent(lr), tables, grads, indexers):
 *   table_t[r] -= lr * sum_{(b,k): idx_t[b*lookups+k] - base == r} grad[b][grad_offset + t*dim + :]
 * Default: deterministic (sum in ascending position order per unique row, one
 * read-modify-write per unique row); builds the indexer from `indices` first unless
 * DLRM_UPDATE_PREBUILT.  DLRM_UPDATE_ATOMIC ignores the indexer (may be NULL). */
int dlrm_sgd_update(dlrm_ctx* ctx, dlrm_tables* tables, dlrm_indexer* indexer, unsigned flags,
                    const void* indices, int itype, int64_t table_stride, int index_base,
                    int batch, int lookups,
                    const void* grad, int grad_dtype, int64_t grad_ld, int64_t grad_offset,
                    float lr);

/* ---- training step: fused forms of the four operators --------------------------------
 * One train! iteration of the sparse half of the model (src/train/train.jl:215-227 and
 * custom_update! :283-290) on one-hot lookups, as two launching calls with the tables
 * unchanged between them:
 *
 * dlrm_step_fwd = dlrm_lookup_interact_fwd(ys = NULL) + dlrm_indexer_build, in one launch
 *   where the shape allows (F <= 32, batch <= 2048): the indexer's workgroups sort while the
 *   gather streams.  `out` is bit-identical to dlrm_lookup_interact_fwd's.  The indexer is
 *   built in "split" form: rows hit by exactly one position of the batch are flagged for the
 *   backward instead of listed for the apply.  dlrm_sgd_update(PREBUILT) with such an indexer
 *   updates the flagged rows too -- unless dlrm_step_bwd's backward (DLRM_STEP_BWD_ONLY or flags 0)
 *   already has, in which case it updates only the repeated rows from their dt rows, so every row
 *   is stepped exactly once whichever call follows the backward.
 * dlrm_step_bwd = dlrm_interact_bwd_gather + dlrm_sgd_update(Descent(lr), PREBUILT) with that
 *   indexer.  dx is bit-identical to dlrm_interact_bwd_gather's and the tables end up
 *   bit-identical to dlrm_sgd_update's result: a once-hit row gets w = fmaf(-lr, g, w) inside
 *   the backward (no other sample reads it), so its dt row is never written or read back;
 *   dt holds only the rows the apply launch reads (x rows and rows of repeated table rows).
 *   dx and dt must be 16-B aligned with leading dimensions divisible by 4.
 *   flags: 0 runs both launches; DLRM_STEP_BWD_ONLY then DLRM_STEP_APPLY_ONLY run them one at a
 *   time (e.g. the apply on another stream, or timed alone). */
#define DLRM_STEP_BWD_ONLY 1u   /* the backward launch only (dx, dt, once-hit rows)       */
#define DLRM_STEP_APPLY_ONLY 2u /* the apply of repeated rows only (reads dt)             */
int dlrm_step_fwd(dlrm_ctx* ctx, const dlrm_tables* tables, dlrm_indexer* indexer,
                  const void* indices, int itype, int64_t table_stride, int index_base, int batch,
                  const void* x, int64_t x_ld, void* out, int64_t out_ld, int padding);
int dlrm_step_bwd(dlrm_ctx* ctx, dlrm_tables* tables, dlrm_indexer* indexer,
                  const void* indices, int itype, int64_t table_stride, int index_base, int batch,
                  const void* x, int64_t x_ld, const void* dout, int64_t dout_ld, int padding,
                  float* dx, int64_t dx_ld, float* dt, int64_t dt_ld, float lr, unsigned flags);
/* Pipelined step: dlrm_step_bwd (flags 0) whose apply launch also builds the NEXT batch's split
 * indexer into next_indexer (same itype / table_stride / index_base / batch as this batch), as
 * extra workgroups of that launch; the next dlrm_step_fwd with next_indexer and next_indices then
 * only gathers (one launch without the indexer's workgroups).  Tables and results are identical to
 * the unpipelined step.  Shapes whose forward has no in-launch indexer (batch > 2048, F > 32, rows
 * not 16-B aligned) run the plain dlrm_step_bwd and leave next_indexer to the next forward.
 * next_indices must hold the next batch when the apply runs (stream order).  flags as
 * dlrm_step_bwd's (the next build rides on the DLRM_STEP_APPLY_ONLY launch).
 * Whether dlrm_step_fwd only gathers is decided on the host when it is called (the indexer holds
 * these indices, prepared): a hipGraph captured from a pipelined sequence is valid only when it is
 * replayed from the indexer state it was captured in (e.g. re-prime before each replayed run). */
int dlrm_step_bwd_prepare(dlrm_ctx* ctx, dlrm_tables* tables, dlrm_indexer* indexer,
                          const void* indices, int itype, int64_t table_stride, int index_base, int batch,
                          const void* x, int64_t x_ld, const void* dout, int64_t dout_ld, int padding,
                          float* dx, int64_t dx_ld, float* dt, int64_t dt_ld, float lr,
                          dlrm_indexer* next_indexer, const void* next_indices, unsigned flags);

/* ---- table-sharded exchange over RCCL ------------------------------------
 * DLRM.jl is one process: maplookup hands its output straight to the interaction (model.jl:161-163).
 * With the tables sharded by table over the GPUs of a node (one host process per GPU), that hand-off
 * is an all-to-all each way.  table_counts[p] = tables owned by rank p (host array, nranks entries);
 * B = samples per rank; blocks are contiguous and in owner order (exchange layout of
 * dlrm_maplookup_blocked / dlrm_scatter_rows):
 *   dlrm_alltoall_fwd: send [nranks][T_me][B][dim] (dtype) -> recv [src][T_src][B][dim]
 *   dlrm_alltoall_bwd: gsend [owner][B][T_owner][dim] (fp32) -> grecv [src][B][T_me][dim]
 *                      (= the [nranks*B][T_me*dim] gradient of this rank's tables for the global batch)
 * dlrm_comm_unique_id fills DLRM_COMM_ID_BYTES bytes on one rank; the caller hands them to every
 * rank (e.g. Julia's Distributed, MPI or a file), which calls dlrm_comm_init with its rank.  Both
 * exchanges are asynchronous on the ctx stream (RCCL group of one send + one receive per peer). */
#define DLRM_COMM_ID_BYTES 128
typedef struct dlrm_comm dlrm_comm;
int dlrm_comm_unique_id(void* id);
int dlrm_comm_init(dlrm_ctx* ctx, const void* id, int rank, int nranks, dlrm_comm** out);
int dlrm_comm_destroy(dlrm_comm* comm);
/* the rank count RCCL reports for the communicator (ncclCommCount), into *nranks */
int dlrm_comm_count(const dlrm_comm* comm, int* nranks);
int dlrm_alltoall_fwd(dlrm_ctx* ctx, dlrm_comm* comm, int dtype, int dim, int batch_local, const int* table_counts,
                      const void* send, void* recv);
int dlrm_alltoall_bwd(dlrm_ctx* ctx, dlrm_comm* comm, int dim, int batch_local, const int* table_counts,
                      const float* gsend, float* grecv);

/* ---- dense half of the training step (the GEMMs stay on hipBLASLt) --------
 * dlrm_bce_head: one launch for the top MLP's head after its last GEMM, replacing
 *   Flux.sigmoid (model.jl:83-89), bce_loss (train.jl:33-41) and rrule(bce_loss) (train.jl:43-64):
 *   prob[b] = sigmoid(logits[b * logits_ld]); *loss = mean(-y·max(log p, -100) + (y-1)·max(log(1-p), -100));
 *   dlogit[b] = (1/B)·((1-y)/(1-p+eps) - y/(p+eps)) · p(1-p);  *dbias (may be NULL) = Σ_b dlogit[b].
 *   fp32; deterministic (fixed reduction order).  batch >= 1.
 * dlrm_relu_bwd_bias: the Dense(relu) pullback seam (model.jl:72-93): g[b][:] *= (y[b][:] > 0)
 *   in place, dbias[n] = Σ_b g[b][n] (two launches: mask + 16-row column sums, then the column
 *   sums of those in chunk order).  work / counters: caller-owned scratch sized by
 *   dlrm_relu_bwd_bias_workspace (counters zeroed once by the caller; the kernel leaves them 0).
 *   n % 4 == 0, y, g 16-B aligned, leading dimensions % 4 == 0.  Deterministic. */
int dlrm_bce_head(dlrm_ctx* ctx, int batch, const float* logits, int64_t logits_ld, const float* labels,
                  float* prob, float* dlogit, float* loss, float* dbias);
int dlrm_relu_bwd_bias_workspace(int batch, int n, int64_t* work_floats, int64_t* counters);
int dlrm_relu_bwd_bias(dlrm_ctx* ctx, int batch, int n, const float* y, int64_t y_ld, float* g, int64_t g_ld,
                       float* dbias, float* work, unsigned* counters);

/* ---- Criteo DAC data path (SURVEY §8 rows f2 + f4; criteo.jl:85-344) ----------------------
 * dlrm_dac_record: DACRecord (criteo.jl:91-95), 160 bytes, the binary file format (mmap-able).
 * dlrm_dac_parse_tsv: parseline over a buffer of TSV lines (criteo.jl:164-176): label Int32,
 *   13 x logtransform(emptyparse(Int32, base 10)) as Float32, 26 x emptyparse(UInt32, base 16).
 *   Blank lines are skipped; *count = records written.  DLRM_E_NOMEM if more than cap lines,
 *   DLRM_E_ARG on a malformed line.  Host only.
 * dlrm_dac_maps_*: categorical_values + reindex/reindex! (criteo.jl:182-262): per feature, ids
 *   1, 2, ... in first-appearance order, accumulated over shards added in order.  Host only.
 * dlrm_dac_reindex: reindex!(data, maps) in place (criteo.jl:251-259); DLRM_E_INDEX for a value
 *   that is not in the maps (the reference's KeyError).
 * dlrm_dac_decode: load! (criteo.jl:284-307) on the device: `batch` contiguous records already in
 *   HBM -> labels [batch] f32, dense [batch][13] f32 (row stride dense_ld), sparse [26][batch]
 *   indices (itype DLRM_I32 / DLRM_I64, table stride table_stride) = DACLoader's
 *   Matrix{UInt32}(B, 26) layout, which is the hot path's [T][B] index layout (index_base 1). */
typedef struct {
    int32_t label;
    float continuous[13];
    uint32_t categorical[26];
} dlrm_dac_record;
typedef struct dlrm_dac_maps dlrm_dac_maps;
int dlrm_dac_parse_tsv(const char* text, int64_t len, dlrm_dac_record* out, int64_t cap, int64_t* count);
int dlrm_dac_maps_create(dlrm_dac_maps** out);
int dlrm_dac_maps_destroy(dlrm_dac_maps* maps);
int dlrm_dac_maps_add(dlrm_dac_maps* maps, const dlrm_dac_record* records, int64_t count);
int dlrm_dac_maps_sizes(const dlrm_dac_maps* maps, int64_t* sizes /* [26] */);
int dlrm_dac_maps_lookup(const dlrm_dac_maps* maps, int feature, uint32_t value, uint32_t* id);
int dlrm_dac_reindex(const dlrm_dac_maps* maps, dlrm_dac_record* records, int64_t count);
int dlrm_dac_decode(dlrm_ctx* ctx, const dlrm_dac_record* records, int batch, float* labels, float* dense,
                    int64_t dense_ld, void* sparse, int itype, int64_t table_stride);
/* Native prefetching DACLoader.  create: `records` (host, count records, kept alive by the
 * caller) and the caller's two output slots (device: labels[k] [batch] f32, dense[k] [batch][13]
 * f32, sparse[k] [26][batch] of itype).  start: one epoch of count/batch whole batches on a
 * native worker thread (pinned staging, upload + dlrm_dac_decode on the loader's own stream).
 * next: blocks until the next batch is decoded, makes consumer_stream wait for it, returns its
 * slot (-1: epoch over).  release: the caller's work on that slot is queued on consumer_stream;
 * the slot may be refilled after it.  stop: ends the epoch early.  start returns DLRM_E_STATE
 * while a slot of the previous epoch is still held (next without release).  The calls for one
 * loader come from one host thread. */
typedef struct dlrm_dac_loader dlrm_dac_loader;
int dlrm_dac_loader_create(int device, const dlrm_dac_record* records, int64_t count, int batch, int itype,
                           float* const* labels, float* const* dense, void* const* sparse, dlrm_dac_loader** out);
int dlrm_dac_loader_start(dlrm_dac_loader* loader, int64_t* nbatches);
int dlrm_dac_loader_next(dlrm_dac_loader* loader, void* consumer_stream, int* slot);
int dlrm_dac_loader_release(dlrm_dac_loader* loader, int slot, void* consumer_stream);
int dlrm_dac_loader_stop(dlrm_dac_loader* loader);
int dlrm_dac_loader_destroy(dlrm_dac_loader* loader);

#ifdef __cplusplus
}
#endif
#endif /* DLRM_HIP_H */
