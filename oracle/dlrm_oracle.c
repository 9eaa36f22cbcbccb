/*
 * dlrm_oracle.c — CPU restatement of darchr/DLRM.jl's embedding + interaction hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/ as the parity checker, by
 * __graft_entry__.smoke() as the checker, and by bench.py's `cpu_baseline` leg (timed,
 * labelled "port": it is a C restatement, not the Julia reference, which cannot run here —
 * no julia binary and its EmbeddingTables/OneDNN path dependencies are absent).
 * The product path (dlrm.jl_amd) never links, loads or calls this file.
 *
 * Pinned by: tests/golden/pytorch_reference_{single,multi}.npz (extracted from the
 * reference HDF5 files under ref/ by tests/golden/make_fixtures.py) and the known-answer vectors of
 * test/model/model.jl and test/model/interact.jl (tests/golden/kat_reference_tests.json).
 *
 * Every function follows the reference algorithm it cites; threading mirrors the
 * reference's Polyester/@threads decomposition (per sample for the interaction, per table
 * for the update), with OpenMP threads instead of Julia tasks.
 *
 * Layout: C row-major, i.e. a Julia (D, N) matrix is [N][D] here.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OK 0
#define E_ARG (-1)
#define E_INDEX (-3)

static inline float bf16_to_f32(uint16_t h) {
    union { uint32_t u; float f; } v;
    v.u = ((uint32_t)h) << 16;
    return v.f;
}

/* round-to-nearest-even, NaN stays NaN */
static inline uint16_t f32_to_bf16(float f) {
    union { uint32_t u; float f; } v;
    v.f = f;
    if ((v.u & 0x7f800000u) == 0x7f800000u && (v.u & 0x007fffffu)) return (uint16_t)((v.u >> 16) | 0x40);
    uint32_t r = v.u + 0x7fffu + ((v.u >> 16) & 1u);
    return (uint16_t)(r >> 16);
}

static inline float ld(const void* p, int dtype, int64_t i) {
    return dtype == 0 ? ((const float*)p)[i] : bf16_to_f32(((const uint16_t*)p)[i]);
}
static inline void st(void* p, int dtype, int64_t i, float v) {
    if (dtype == 0) ((float*)p)[i] = v;
    else ((uint16_t*)p)[i] = f32_to_bf16(v);
}

static void set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/*
 * maplookup(PreallocationStrategy(out_offset), tables, sparse)
 * (EmbeddingTables, un-vendored; call site src/model/model.jl:161; semantics pinned by
 * test/model/embedding_update.jl:23-33: maplookup == mapreduce(lookup, vcat); pooled
 * multi-hot is a SUM over the L x B index matrix, sample-major, criteo.jl:551-557 —
 * confirmed against pytorch_reference_multi.hdf5 `concatenated_result`).
 * Rows [0, out_offset) of each output column are left untouched (interact.jl:264-270).
 */
int oracle_maplookup(int T, int D, int dtype, const void* const* tables, const int64_t* nrows,
                     const int64_t* idx, int64_t tstride, int base, int B, int L,
                     void* out, int64_t out_ld, int64_t out_offset, int nthreads) {
    if (T < 0 || D <= 0 || B < 0 || L <= 0) return E_ARG;
    /* BoundsError before any write, as Julia's checked indexing would raise */
    for (int t = 0; t < T; ++t)
        for (int64_t p = 0; p < (int64_t)B * L; ++p) {
            int64_t r = idx[t * tstride + p] - base;
            if (r < 0 || r >= nrows[t]) return E_INDEX;
        }
    set_threads(nthreads);
    int64_t total = (int64_t)T * B;
#pragma omp parallel for schedule(static)
    for (int64_t it = 0; it < total; ++it) {
        int b = (int)(it / T), t = (int)(it % T);
        float acc[1024];
        float* a = D <= 1024 ? acc : (float*)malloc(sizeof(float) * D);
        /* first row seeds the sum (so L = 1 is an exact copy, -0.0 included), then k order */
        int64_t r0 = idx[t * tstride + (int64_t)b * L] - base;
        for (int c = 0; c < D; ++c) a[c] = ld(tables[t], dtype, r0 * D + c);
        for (int k = 1; k < L; ++k) {
            int64_t r = idx[t * tstride + (int64_t)b * L + k] - base;
            for (int c = 0; c < D; ++c) a[c] += ld(tables[t], dtype, r * D + c);
        }
        for (int c = 0; c < D; ++c) st(out, dtype, (int64_t)b * out_ld + out_offset + (int64_t)t * D + c, a[c]);
        if (a != acc) free(a);
    }
    return OK;
}

/*
 * (dot::DotInteraction)(x, ys) — src/model/interact.jl:394-411.
 *   fast_vcat (:271-281): ys[b][0:d] = x[b]
 *   process_batches (:449-467) -> process_slice! (:338-362) per sample, threaded over B:
 *     dst[0:d] = x ; gemmavx!(scratch, T', T) (:318-326, k ascending, fp32 scratch even for
 *     bf16 inputs since DotInteraction's scratchpads are Float32, criteo.jl:420) ;
 *     triangular_slice_kernel! (:64-75): for i = 1..F-1, j = 0..i-1: Z[i][j] ; zero padding.
 */
int oracle_interact_fwd(int dtype, int d, int F, int B, const void* x, int64_t x_ld,
                        void* ys, int64_t ys_ld, void* out, int64_t out_ld, int padding,
                        int nthreads) {
    if (d <= 0 || F <= 0 || B < 0 || padding < 0) return E_ARG;
    set_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < B; ++b) {
        for (int c = 0; c < d; ++c) st(ys, dtype, (int64_t)b * ys_ld + c, ld(x, dtype, (int64_t)b * x_ld + c));
        for (int c = 0; c < d; ++c) st(out, dtype, (int64_t)b * out_ld + c, ld(x, dtype, (int64_t)b * x_ld + c));
        int64_t o = (int64_t)b * out_ld + d;
        const int64_t tb = (int64_t)b * ys_ld;
        for (int i = 1; i < F; ++i)
            for (int j = 0; j < i; ++j) {
                float z = 0.0f;
                for (int c = 0; c < d; ++c)
                    z = fmaf(ld(ys, dtype, tb + (int64_t)i * d + c), ld(ys, dtype, tb + (int64_t)j * d + c), z);
                st(out, dtype, o++, z);
            }
        for (int p = 0; p < padding; ++p) st(out, dtype, o++, 0.0f);
    }
    return OK;
}

/*
 * dot_back / process_batches_back — src/model/interact.jl:415-489.
 *   triangular_slice_back_fuse_add_transpose_kernel! (:154-173): S symmetric, zero diagonal
 *   gemmavx!(vdt, vt, scratch) (:486): dt[f][c] = sum_j T[j][c] * S[j][f]  (j ascending)
 *   sumavx(dx1, dx2) (:434): dx = dout[0:d] + dt[0][0:d]
 * bf16 dout is converted to fp32 first (:419-422) and dt is fp32 (similar(Δ, Float32)).
 */
int oracle_interact_bwd(int dtype, int d, int F, int B, const void* dout, int64_t dout_ld,
                        int padding, const void* t, int64_t t_ld, float* dx, int64_t dx_ld,
                        float* dt, int64_t dt_ld, int nthreads) {
    (void)padding;
    if (d <= 0 || F <= 0 || B < 0) return E_ARG;
    set_threads(nthreads);
#pragma omp parallel
    {
        float* S = (float*)malloc(sizeof(float) * F * F);
#pragma omp for schedule(static)
        for (int b = 0; b < B; ++b) {
            const int64_t ob = (int64_t)b * dout_ld + d;
            for (int i = 0; i < F; ++i)
                for (int j = 0; j < F; ++j) {
                    float v = 0.0f;
                    if (i > j) v = ld(dout, dtype, ob + (int64_t)i * (i - 1) / 2 + j);
                    else if (i < j) v = ld(dout, dtype, ob + (int64_t)j * (j - 1) / 2 + i);
                    S[i * F + j] = v;
                }
            const int64_t tb = (int64_t)b * t_ld;
            for (int f = 0; f < F; ++f)
                for (int c = 0; c < d; ++c) {
                    float acc = 0.0f;
                    for (int j = 0; j < F; ++j) acc = fmaf(ld(t, dtype, tb + (int64_t)j * d + c), S[j * F + f], acc);
                    dt[(int64_t)b * dt_ld + (int64_t)f * d + c] = acc;
                }
            for (int c = 0; c < d; ++c)
                dx[(int64_t)b * dx_ld + c] = ld(dout, dtype, (int64_t)b * dout_ld + c) + dt[(int64_t)b * dt_ld + c];
        }
        free(S);
    }
    return OK;
}

typedef struct { int64_t row; int64_t pos; } rp_t;
static int rp_cmp(const void* a, const void* b) {
    const rp_t* x = (const rp_t*)a;
    const rp_t* y = (const rp_t*)b;
    if (x->row != y->row) return x->row < y->row ? -1 : 1;
    return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

/*
 * EmbeddingTables.update!(Descent(lr), tables, grads, indexers; num_splits, nthreads)
 * (un-vendored; call src/train/train.jl:274-292, checked by src/validation.jl:125-146):
 * the maplookup pullback gives, per table, SparseEmbeddingUpdate(delta = dt rows of table t,
 * indices) (test/model/embedding_update.jl:35-40); update! dedupes the indices through a
 * SparseIndexer and applies row .-= lr * (sum of the delta columns hitting that row), a
 * pooled bag broadcasting its sample's delta to each of its L lookups.  Verified against
 * `update_emb_*` of both golden files (tests/golden/fixtures_meta.json).
 * Threaded across tables (the reference splits tables over `nthreads` update tasks).
 * unique_counts[t] (optional) receives the number of distinct rows touched in table t.
 */
int oracle_sgd_update(int T, int D, int dtype, void* const* tables, const int64_t* nrows,
                      const int64_t* idx, int64_t tstride, int base, int B, int L,
                      const void* grad, int grad_dtype, int64_t grad_ld, int64_t grad_offset,
                      float lr, int64_t* unique_counts, int nthreads) {
    if (T < 0 || D <= 0 || B < 0 || L <= 0) return E_ARG;
    for (int t = 0; t < T; ++t)
        for (int64_t p = 0; p < (int64_t)B * L; ++p) {
            int64_t r = idx[t * tstride + p] - base;
            if (r < 0 || r >= nrows[t]) return E_INDEX;
        }
    set_threads(nthreads);
    const int64_t N = (int64_t)B * L;
#pragma omp parallel
    {
        rp_t* rp = (rp_t*)malloc(sizeof(rp_t) * (N > 0 ? N : 1));
        float* acc = (float*)malloc(sizeof(float) * D);
#pragma omp for schedule(dynamic, 1)
        for (int t = 0; t < T; ++t) {
            for (int64_t p = 0; p < N; ++p) {
                rp[p].row = idx[t * tstride + p] - base;
                rp[p].pos = p;
            }
            qsort(rp, (size_t)N, sizeof(rp_t), rp_cmp);
            int64_t uniq = 0;
            for (int64_t s = 0; s < N;) {
                int64_t e = s;
                for (int c = 0; c < D; ++c) acc[c] = 0.0f;
                while (e < N && rp[e].row == rp[s].row) {
                    int64_t b = rp[e].pos / L;
                    for (int c = 0; c < D; ++c)
                        acc[c] += ld(grad, grad_dtype, b * grad_ld + grad_offset + (int64_t)t * D + c);
                    ++e;
                }
                int64_t r = rp[s].row;
                for (int c = 0; c < D; ++c) {
                    float w = ld(tables[t], dtype, r * D + c);
                    st(tables[t], dtype, r * D + c, fmaf(-lr, acc[c], w));
                }
                ++uniq;
                s = e;
            }
            if (unique_counts) unique_counts[t] = uniq;
        }
        free(acc);
        free(rp);
    }
    return OK;
}

/* triangular_slice_kernel! (:64-75) on one row-major F x F matrix (tests of the KAT). */
void oracle_triangular_slice(int F, const float* z, float* y) {
    int64_t o = 0;
    for (int i = 1; i < F; ++i)
        for (int j = 0; j < i; ++j) y[o++] = z[i * F + j];
}

/* triangular_slice_back_fuse_add_transpose_kernel! (:154-173) */
void oracle_triangular_slice_back_sym(int F, const float* y, float* z) {
    for (int i = 0; i < F; ++i)
        for (int j = 0; j < F; ++j) {
            if (i == j) z[i * F + j] = 0.0f;
            else if (i > j) z[i * F + j] = y[(int64_t)i * (i - 1) / 2 + j];
            else z[i * F + j] = y[(int64_t)j * (j - 1) / 2 + i];
        }
}

/* CPU-baseline harness helper: fills n floats with U(lo, hi) from a counter-based
 * splitmix64 stream (deterministic for any thread count). */
void oracle_fill_uniform(float* p, int64_t n, float lo, float hi, uint64_t seed, int nthreads) {
    set_threads(nthreads);
    const float scale = (hi - lo) / 16777216.0f;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = lo + (float)(z >> 40) * scale;
    }
}
