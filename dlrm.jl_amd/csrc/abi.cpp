// abi.cpp — the extern "C" boundary declared in include/dlrm_hip.h.
//
// Owns the three handle types (ctx, tables, indexer), validates arguments on the host,
// maps HIP errors to dlrm_status codes and forwards to the kernel launchers.  No launching
// entry point allocates or synchronises (hipGraph-capturable).
#include <dlfcn.h>
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <unistd.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "common.hpp"
#include "apply.hpp"

using namespace dlrm;

struct dlrm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // side stream + fork/join events: work that depends only on the indices (the hash indexer
    // build) runs beside the forward; graph capture follows the fork and the join
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    unsigned* err = nullptr;  // device error word
    // host-visible copy of it (pinned), refreshed by dlrm_error_snapshot on the stream and read by
    // dlrm_error_peek without touching the GPU: bounds errors of deferred work reach the host
    // without a per-step synchronisation
    volatile unsigned* err_host = nullptr;
    int cus = 256;
    char msg[512] = {0};
};

struct dlrm_tables {
    dlrm_ctx* ctx = nullptr;
    int T = 0, D = 0, dtype = 0;
    TableDesc* d_desc = nullptr;
    std::vector<TableDesc> h_desc;
    bool aligned16 = true;
};

struct dlrm_indexer {
    dlrm_ctx* ctx = nullptr;
    int T = 0;
    int parts_log2 = 0;  // the wave builds of <= 2048 positions per table: log2 parts (0: the default, 16)
    int TV = 0;  // tables of the per-table arrays: 4T when the forward launch may split tables by row bits
    IndexerDev dev{};
    void* block = nullptr;  // one allocation for every array
    size_t bytes = 0;       // its size
    void* partial_big = nullptr;  // partial rows for D > kPartialDim (allocated on first use)
    // recorded by the last build
    bool built = false;
    bool split = false;  // built by dlrm_step_fwd's kernel: once-hit rows are left to the backward
    bool prepared = false;  // built by dlrm_step_bwd_prepare for the next dlrm_step_fwd (not yet consumed)
    bool singles_done = false;  // a split backward has applied this build's once-hit rows already
    // device words for the bounds errors of builds that may run beside a step's write-deciding
    // kernels, which read the ctx's flag to decide whether to write (raising there would be a race,
    // ADVICE r5): [0] dlrm_indexer_prepare (a side-stream build beside the current step; cleared
    // before each build, folded into the ctx's flag by the apply of this indexer), [1] the NEXT
    // batch's build inside an apply launch (dlrm_step_bwd_prepare; nothing reads it).  Either way the
    // forward / lookup of the same indices raises their errors on the ctx's flag.
    unsigned* prep_err = nullptr;
    const void* indices = nullptr;
    int itype = 0, base = 0, B = 0, L = 0;
    int64_t tstride = 0;
};

namespace dlrm {
unsigned* ctx_error_word(dlrm_ctx* ctx) { return ctx->err; }
hipStream_t ctx_stream(dlrm_ctx* ctx) { return ctx->stream; }
int ctx_num_cus(dlrm_ctx* ctx) { return ctx->cus; }
static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
const Knobs& knobs() {
    static const Knobs k{env_int("DLRM_STEP_PARTS", 0),       env_int("DLRM_BUILD_PARTS", 0),
                         env_int("DLRM_RELU_2PASS", 1) == 0, env_int("DLRM_BWD_YS", 1) == 0,
                         env_int("DLRM_BWD_SPLIT", 1) == 0,  env_int("DLRM_BWD_SPB", 0),
                         env_int("DLRM_BWD_CPL", 0),         env_int("DLRM_UPD_SBU", 1),
                         env_int("DLRM_WAVE_ROUNDS", 0),     env_int("DLRM_BAG_WAVE", 1) == 0,
                         env_int("DLRM_BAG_VS", 0),          env_int("DLRM_BAG_SPLIT", 1)};
    return k;
}
int ctx_device(dlrm_ctx* ctx) { return ctx->device; }
int ctx_fail(dlrm_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(ctx->msg, sizeof(ctx->msg), fmt, ap);
        va_end(ap);
    }
    return code;
}
int ctx_hip(dlrm_ctx* ctx, hipError_t e, const char* what) {
    if (e == hipSuccess) return DLRM_OK;
    return ctx_fail(ctx, e == hipErrorOutOfMemory ? DLRM_E_NOMEM : DLRM_E_HIP, "%s: %s", what, hipGetErrorString(e));
}
}  // namespace dlrm

#define CHECK_ARG(cond, ...) \
    do {                     \
        if (!(cond)) return ctx_fail(ctx, DLRM_E_ARG, __VA_ARGS__); \
    } while (0)

static int hip_set(dlrm_ctx* ctx) { return ctx_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice"); }

// parts per table of the step's split indexer build (DLRM_STEP_PARTS = 1, 2, 4 or 8 overrides,
// for comparison).  Measured (profiles/r3m_*): inside the step forward 4 parts (8 add more
// workgroups than they save in sort depth beside the D = 128 gather); inside the apply launch
// for rows of <= 256 B 8 parts (D = 16: apply + build 12.8 -> 11.4 us), for fp32 x 128 4.
static int step_parts_log2(int dflt = kStepParts) {
    const int forced = knobs().step_parts;
    const int p = forced > 0 ? forced : dflt;
    return p >= 32 ? 5 : (p >= 16 ? 4 : (p >= 8 ? 3 : (p >= 4 ? 2 : (p >= 2 ? 1 : 0))));
}

// vshift of the wave build of `batch` positions per table (the step forward's in-launch build and
// the in-apply / prepared builds): 16 parts per table up to 2048 positions (DLRM_STEP_PARTS may force
// fewer, >= 4), then 16 parts per 2048 positions (wave_vshift)
static int wave_parts_log2(int64_t batch, const dlrm_indexer* ix = nullptr) {
    if (batch > kStepIndexMaxN) return wave_vshift(batch);
    if (ix && ix->parts_log2 && !knobs().step_parts) return ix->parts_log2;  // (dlrm_indexer_set_parts)
    const int vs = step_parts_log2(kWaveBuildParts);
    return vs < 2 ? 2 : vs;
}

static bool has_parts(const dlrm_indexer* ix, int vs) { return (int64_t)ix->TV >= ((int64_t)ix->T << vs) && ix->T > 0; }

static void record_build(dlrm_indexer* ix, bool split, const void* indices, int itype, int64_t tstride, int base,
                         int B, int L) {
    ix->built = true;
    ix->split = split;
    ix->prepared = false;
    ix->singles_done = false;
    ix->dev.has_map = 0;  // (set by dlrm_step_bwd_prepare, whose wave build writes the item map)
    ix->dev.build_err = nullptr;  // (set by dlrm_indexer_prepare)
    ix->indices = indices;
    ix->itype = itype;
    ix->tstride = tstride;
    ix->base = base;
    ix->B = B;
    ix->L = L;
}

static bool built_from(const dlrm_indexer* ix, const void* indices, int itype, int64_t tstride, int base, int B,
                       int L) {
    return ix->built && ix->indices == indices && ix->B == B && ix->L == L && ix->itype == itype &&
           ix->tstride == tstride && ix->base == base;
}

static int ensure_side(dlrm_ctx* ctx) {
    if (ctx->side) return DLRM_OK;
    int rc = ctx_hip(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking), "hipStreamCreate(side)");
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming), "hipEventCreate");
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming), "hipEventCreate");
    return rc;
}

extern "C" {

int dlrm_abi_version(void) { return DLRM_HIP_ABI_VERSION; }

int dlrm_ctx_create(int device, void* stream, dlrm_ctx** out) {
    if (!out) return DLRM_E_ARG;
    *out = nullptr;
    dlrm_ctx* ctx = new (std::nothrow) dlrm_ctx();
    if (!ctx) return DLRM_E_NOMEM;
    ctx->device = device;
    ctx->stream = (hipStream_t)stream;
    int rc = hip_set(ctx);
    if (rc == DLRM_OK) {
        hipDeviceProp_t prop;
        rc = ctx_hip(ctx, hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
        if (rc == DLRM_OK) ctx->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    }
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipMalloc((void**)&ctx->err, 16), "hipMalloc(err)");
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipMemset(ctx->err, 0, 16), "hipMemset(err)");
    if (rc == DLRM_OK) {
        void* h = nullptr;
        rc = ctx_hip(ctx, hipHostMalloc(&h, 64, hipHostMallocMapped), "hipHostMalloc(err_host)");
        if (rc == DLRM_OK) {
            memset(h, 0, 64);
            ctx->err_host = (volatile unsigned*)h;
            void* dh = nullptr;  // its device address, kept in the error word's second half
            rc = ctx_hip(ctx, hipHostGetDevicePointer(&dh, h, 0), "hipHostGetDevicePointer(err_host)");
            if (rc == DLRM_OK)
                rc = ctx_hip(ctx, hipMemcpy((char*)ctx->err + 8, &dh, sizeof(dh), hipMemcpyHostToDevice),
                             "write err_host address");
        }
    }
    if (rc != DLRM_OK) {
        if (ctx->err) (void)hipFree(ctx->err);
        if (ctx->err_host) (void)hipHostFree((void*)ctx->err_host);
        delete ctx;
        return rc;
    }
    *out = ctx;
    return DLRM_OK;
}

int dlrm_ctx_destroy(dlrm_ctx* ctx) {
    if (!ctx) return DLRM_OK;
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->err) (void)hipFree(ctx->err);
    if (ctx->err_host) (void)hipHostFree((void*)ctx->err_host);
    delete ctx;
    return DLRM_OK;
}

int dlrm_ctx_set_stream(dlrm_ctx* ctx, void* stream) {
    if (!ctx) return DLRM_E_ARG;
    ctx->stream = (hipStream_t)stream;
    return DLRM_OK;
}

const char* dlrm_last_error(const dlrm_ctx* ctx) { return ctx ? ctx->msg : "null context"; }

int dlrm_sync(dlrm_ctx* ctx) {
    if (!ctx) return DLRM_E_ARG;
    return ctx_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
}

int dlrm_check_bounds(dlrm_ctx* ctx) {
    if (!ctx) return DLRM_E_ARG;
    unsigned h = 0;
    int rc = ctx_hip(ctx, hipMemcpyAsync(&h, ctx->err, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream),
                     "read error word");
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipMemsetAsync(ctx->err, 0, sizeof(unsigned), ctx->stream), "clear error word");
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if (rc != DLRM_OK) return rc;
    ctx->err_host[0] = 0;  // (the flag is clear now; a stale snapshot must not report it again)
    if (h & kErrIndex) return ctx_fail(ctx, DLRM_E_INDEX, "BoundsError: an embedding index was out of range");
    return DLRM_OK;
}

int dlrm_error_snapshot(dlrm_ctx* ctx) {
    if (!ctx) return DLRM_E_ARG;
    return ctx_hip(ctx, hipMemcpyAsync((void*)ctx->err_host, ctx->err, sizeof(unsigned), hipMemcpyDeviceToHost,
                                       ctx->stream),
                   "dlrm_error_snapshot");
}

int dlrm_error_peek(const dlrm_ctx* ctx, unsigned* word) {
    if (!ctx || !word) return DLRM_E_ARG;
    *word = ctx->err_host[0];
    return DLRM_OK;
}

int dlrm_malloc(dlrm_ctx* ctx, size_t bytes, void** dptr) {
    CHECK_ARG(ctx && dptr, "dlrm_malloc: null argument");
    *dptr = nullptr;
    if (bytes == 0) return DLRM_OK;
    return ctx_hip(ctx, hipMalloc(dptr, bytes), "hipMalloc");
}

int dlrm_free(dlrm_ctx* ctx, void* dptr) {
    CHECK_ARG(ctx, "dlrm_free: null ctx");
    if (!dptr) return DLRM_OK;
    return ctx_hip(ctx, hipFree(dptr), "hipFree");
}

int dlrm_memcpy_h2d(dlrm_ctx* ctx, void* dst, const void* src, size_t bytes) {
    CHECK_ARG(ctx && (bytes == 0 || (dst && src)), "dlrm_memcpy_h2d: null argument");
    int rc = ctx_hip(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream), "memcpy h2d");
    return rc ? rc : ctx_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
}

int dlrm_memcpy_h2d_async(dlrm_ctx* ctx, void* dst, const void* src, size_t bytes) {
    CHECK_ARG(ctx && (bytes == 0 || (dst && src)), "dlrm_memcpy_h2d_async: null argument");
    return ctx_hip(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream), "memcpy h2d async");
}

int dlrm_host_register(void* ptr, size_t bytes) {
    if (!ptr || bytes == 0) return DLRM_E_ARG;
    return hipHostRegister(ptr, bytes, hipHostRegisterDefault) == hipSuccess ? DLRM_OK : DLRM_E_HIP;
}

int dlrm_host_unregister(void* ptr) {
    if (!ptr) return DLRM_E_ARG;
    return hipHostUnregister(ptr) == hipSuccess ? DLRM_OK : DLRM_E_HIP;
}

int dlrm_memcpy_d2h(dlrm_ctx* ctx, void* dst, const void* src, size_t bytes) {
    CHECK_ARG(ctx && (bytes == 0 || (dst && src)), "dlrm_memcpy_d2h: null argument");
    int rc = ctx_hip(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream), "memcpy d2h");
    return rc ? rc : ctx_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
}

// ---------------------------------------------------------------------------- tables
int dlrm_tables_create(dlrm_ctx* ctx, int num_tables, int dim, int dtype, void* const* data, const int64_t* nrows,
                       dlrm_tables** out) {
    CHECK_ARG(ctx && out, "dlrm_tables_create: null argument");
    *out = nullptr;
    CHECK_ARG(num_tables >= 0 && dim > 0, "dlrm_tables_create: num_tables=%d dim=%d", num_tables, dim);
    CHECK_ARG(dtype == DLRM_F32 || dtype == DLRM_BF16, "dlrm_tables_create: unknown dtype %d", dtype);
    CHECK_ARG(num_tables == 0 || (data && nrows), "dlrm_tables_create: null data/nrows");
    dlrm_tables* tb = new (std::nothrow) dlrm_tables();
    if (!tb) return DLRM_E_NOMEM;
    tb->ctx = ctx;
    tb->T = num_tables;
    tb->D = dim;
    tb->dtype = dtype;
    tb->h_desc.resize(num_tables);
    for (int t = 0; t < num_tables; ++t) {
        if (nrows[t] < 0 || nrows[t] >= 0xFFFFFFFFll || (nrows[t] > 0 && !data[t])) {
            delete tb;
            return ctx_fail(ctx, DLRM_E_ARG, "dlrm_tables_create: table %d has nrows=%lld", t, (long long)nrows[t]);
        }
        tb->h_desc[t].data = data[t];
        tb->h_desc[t].nrows = nrows[t];
        if ((uintptr_t)data[t] % 16) tb->aligned16 = false;
    }
    int rc = hip_set(ctx);
    if (rc == DLRM_OK && num_tables > 0) {
        rc = ctx_hip(ctx, hipMalloc((void**)&tb->d_desc, sizeof(TableDesc) * num_tables), "hipMalloc(tables)");
        if (rc == DLRM_OK)
            rc = ctx_hip(ctx, hipMemcpy(tb->d_desc, tb->h_desc.data(), sizeof(TableDesc) * num_tables,
                                        hipMemcpyHostToDevice), "hipMemcpy(tables)");
    }
    if (rc != DLRM_OK) {
        if (tb->d_desc) (void)hipFree(tb->d_desc);
        delete tb;
        return rc;
    }
    *out = tb;
    return DLRM_OK;
}

int dlrm_tables_destroy(dlrm_tables* tb) {
    if (!tb) return DLRM_OK;
    if (tb->d_desc) (void)hipFree(tb->d_desc);
    delete tb;
    return DLRM_OK;
}

static int check_indices(dlrm_ctx* ctx, const dlrm_tables* tb, const void* indices, int itype, int64_t tstride,
                         int batch, int lookups) {
    CHECK_ARG(itype == DLRM_I32 || itype == DLRM_I64, "unknown index type %d", itype);
    CHECK_ARG(batch >= 0 && lookups >= 1, "batch=%d lookups=%d", batch, lookups);
    CHECK_ARG((int64_t)batch * lookups < (1ll << 31), "batch*lookups exceeds 2^31");
    CHECK_ARG(batch == 0 || tb->T == 0 || indices, "null indices");
    CHECK_ARG(tb->T <= 1 || tstride >= (int64_t)batch * lookups, "table_stride %lld < batch*lookups %lld",
              (long long)tstride, (long long)batch * lookups);
    return DLRM_OK;
}

int dlrm_maplookup(dlrm_ctx* ctx, const dlrm_tables* tb, const void* indices, int itype, int64_t table_stride,
                   int index_base, int batch, int lookups, void* out, int64_t out_ld, int64_t out_offset) {
    CHECK_ARG(ctx && tb, "dlrm_maplookup: null ctx/tables");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, lookups);
    if (rc) return rc;
    CHECK_ARG(batch == 0 || tb->T == 0 || out, "dlrm_maplookup: null out");
    CHECK_ARG(out_offset >= 0 && out_ld >= out_offset + (int64_t)tb->T * tb->D,
              "dlrm_maplookup: out_ld %lld < out_offset %lld + T*D %lld", (long long)out_ld, (long long)out_offset,
              (long long)tb->T * tb->D);
    return launch_maplookup(ctx, tb->d_desc, tb->aligned16, tb->T, tb->D, tb->dtype, indices, itype, table_stride,
                            index_base, batch, lookups, out, out_ld, out_offset, tb->h_desc.data());
}

int dlrm_maplookup_blocked(dlrm_ctx* ctx, const dlrm_tables* tb, const void* indices, int itype,
                           int64_t table_stride, int index_base, int batch, int lookups, void* out, int64_t out_ld,
                           int64_t out_offset, int64_t out_table_stride, int64_t block_rows, int64_t block_stride) {
    CHECK_ARG(ctx && tb, "dlrm_maplookup_blocked: null ctx/tables");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, lookups);
    if (rc) return rc;
    CHECK_ARG(batch == 0 || tb->T == 0 || out, "dlrm_maplookup_blocked: null out");
    CHECK_ARG(out_ld >= 0 && out_offset >= 0 && out_table_stride >= 0 && block_rows > 0 && block_stride >= 0,
              "dlrm_maplookup_blocked: negative stride or block_rows < 1");
    return launch_maplookup_map(ctx, tb->d_desc, tb->aligned16, tb->T, tb->D, tb->dtype, indices, itype,
                                table_stride, index_base, batch, lookups, out,
                                OutMap{out_ld, out_offset, out_table_stride, block_rows, block_stride},
                                tb->h_desc.data());
}

int dlrm_scatter_rows(dlrm_ctx* ctx, int esize, int num_tables, int batch, int dim, const void* src, int64_t src_ld,
                      int64_t src_offset, void* dst, const int64_t* dst_base, const int64_t* dst_ld) {
    CHECK_ARG(ctx, "dlrm_scatter_rows: null ctx");
    CHECK_ARG(esize == 2 || esize == 4, "dlrm_scatter_rows: esize %d", esize);
    CHECK_ARG(num_tables >= 0 && batch >= 0 && dim >= 0 && src_ld >= 0 && src_offset >= 0,
              "dlrm_scatter_rows: negative size");
    CHECK_ARG(num_tables == 0 || batch == 0 || dim == 0 || (src && dst && dst_base && dst_ld),
              "dlrm_scatter_rows: null buffer");
    // 16-B pieces when the source rows allow (a destination row that is not 16-B aligned is
    // copied element by element on the device)
    const int u = 16 / esize;
    const bool vec = (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0 && src_ld % u == 0 && src_offset % u == 0 &&
                     dim % u == 0;
    return launch_scatter_rows(ctx, esize, num_tables, batch, dim, src, src_ld, src_offset, dst, dst_base, dst_ld,
                               vec);
}

// ---------------------------------------------------------------------- dense seams
int dlrm_bce_head(dlrm_ctx* ctx, int batch, const float* logits, int64_t logits_ld, const float* labels, float* prob,
                  float* dlogit, float* loss, float* dbias) {
    CHECK_ARG(ctx, "dlrm_bce_head: null ctx");
    CHECK_ARG(batch >= 1 && logits_ld >= 1, "dlrm_bce_head: batch=%d logits_ld=%lld", batch, (long long)logits_ld);
    CHECK_ARG(logits && labels && prob && dlogit && loss, "dlrm_bce_head: null buffer");
    return launch_bce_head(ctx, batch, logits, logits_ld, labels, prob, dlogit, loss, dbias);
}

int dlrm_relu_bwd_bias_workspace(int batch, int n, int64_t* work_floats, int64_t* counters) {
    if (batch < 0 || n < 0 || !work_floats || !counters) return DLRM_E_ARG;
    *work_floats = relu_bwd_chunks(batch) * (int64_t)n;
    *counters = relu_bwd_groups(n);
    return DLRM_OK;
}

int dlrm_relu_bwd_bias(dlrm_ctx* ctx, int batch, int n, const float* y, int64_t y_ld, float* g, int64_t g_ld,
                       float* dbias, float* work, unsigned* counters) {
    CHECK_ARG(ctx, "dlrm_relu_bwd_bias: null ctx");
    CHECK_ARG(batch >= 0 && n >= 0 && n % 4 == 0, "dlrm_relu_bwd_bias: batch=%d n=%d (n %% 4 == 0)", batch, n);
    CHECK_ARG(y_ld >= n && g_ld >= n && y_ld % 4 == 0 && g_ld % 4 == 0, "dlrm_relu_bwd_bias: leading dimensions");
    if (batch == 0 || n == 0) return DLRM_OK;
    CHECK_ARG(y && g && dbias && work && counters, "dlrm_relu_bwd_bias: null buffer");
    CHECK_ARG((uintptr_t)y % 16 == 0 && (uintptr_t)g % 16 == 0 && (uintptr_t)dbias % 16 == 0 &&
                  (uintptr_t)work % 16 == 0,
              "dlrm_relu_bwd_bias: buffers must be 16-B aligned");
    return launch_relu_bwd_bias(ctx, batch, n, y, y_ld, g, g_ld, dbias, work, counters);
}

int dlrm_dac_decode(dlrm_ctx* ctx, const dlrm_dac_record* records, int batch, float* labels, float* dense,
                    int64_t dense_ld, void* sparse, int itype, int64_t table_stride) {
    CHECK_ARG(ctx, "dlrm_dac_decode: null ctx");
    CHECK_ARG(batch >= 0 && dense_ld >= 13 && table_stride >= batch, "dlrm_dac_decode: batch=%d dense_ld=%lld "
              "table_stride=%lld", batch, (long long)dense_ld, (long long)table_stride);
    CHECK_ARG(itype == DLRM_I32 || itype == DLRM_I64, "dlrm_dac_decode: itype %d", itype);
    CHECK_ARG(batch == 0 || (records && labels && dense && sparse), "dlrm_dac_decode: null buffer");
    CHECK_ARG((uintptr_t)records % 4 == 0, "dlrm_dac_decode: records must be 4-B aligned");
    return launch_dac_decode(ctx, records, batch, labels, dense, dense_ld, sparse, itype, table_stride);
}

// ---------------------------------------------------------------------- interaction
int dlrm_interact_fwd(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch, const void* x, int64_t x_ld,
                      void* ys, int64_t ys_ld, void* out, int64_t out_ld, int padding) {
    CHECK_ARG(ctx, "dlrm_interact_fwd: null ctx");
    CHECK_ARG(dtype == DLRM_F32 || dtype == DLRM_BF16, "dlrm_interact_fwd: dtype %d", dtype);
    CHECK_ARG(d > 0 && num_features >= 1 && batch >= 0 && padding >= 0, "dlrm_interact_fwd: d=%d F=%d B=%d pad=%d", d,
              num_features, batch, padding);
    const int64_t P = (int64_t)num_features * (num_features - 1) / 2;
    CHECK_ARG(x_ld >= d && ys_ld >= (int64_t)num_features * d && out_ld >= d + P + padding,
              "dlrm_interact_fwd: leading dimensions too small");
    CHECK_ARG(batch == 0 || (x && ys && out), "dlrm_interact_fwd: null buffer");
    return launch_interact_fwd(ctx, dtype, d, num_features, batch, x, x_ld, ys, ys_ld, out, out_ld, padding);
}

int dlrm_lookup_interact_fwd(dlrm_ctx* ctx, const dlrm_tables* tb, const void* indices, int itype,
                             int64_t table_stride, int index_base, int batch, int lookups, const void* x,
                             int64_t x_ld, void* ys, int64_t ys_ld, void* out, int64_t out_ld, int padding) {
    CHECK_ARG(ctx && tb, "dlrm_lookup_interact_fwd: null ctx/tables");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, lookups);
    if (rc) return rc;
    const int d = tb->D, F = tb->T + 1;
    const int64_t P = (int64_t)F * (F - 1) / 2;
    CHECK_ARG(padding >= 0 && x_ld >= d && (!ys || ys_ld >= (int64_t)F * d) && out_ld >= d + P + padding,
              "dlrm_lookup_interact_fwd: leading dimensions too small");
    CHECK_ARG(batch == 0 || (x && out), "dlrm_lookup_interact_fwd: null buffer");
    rc = launch_lookup_interact_fwd(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype, table_stride,
                                    index_base, lookups, d, batch, x, x_ld, ys, ys_ld, out, out_ld, padding, tb->h_desc.data());
    if (rc != DLRM_E_UNSUPPORTED) return rc;
    if (!ys)
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED,
                        "dlrm_lookup_interact_fwd: ys may be NULL only where the fused kernel applies "
                        "(16-B aligned rows, F <= 96)");
    rc = launch_maplookup(ctx, tb->d_desc, tb->aligned16, tb->T, tb->D, tb->dtype, indices, itype, table_stride,
                          index_base, batch, lookups, ys, ys_ld, d, tb->h_desc.data());
    if (rc) return rc;
    return launch_interact_fwd(ctx, tb->dtype, d, F, batch, x, x_ld, ys, ys_ld, out, out_ld, padding);
}

int dlrm_interact_bwd(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch, const void* dout, int64_t dout_ld,
                      int padding, const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld) {
    CHECK_ARG(ctx, "dlrm_interact_bwd: null ctx");
    CHECK_ARG(dtype == DLRM_F32 || dtype == DLRM_BF16, "dlrm_interact_bwd: dtype %d", dtype);
    CHECK_ARG(d > 0 && num_features >= 1 && batch >= 0 && padding >= 0, "dlrm_interact_bwd: d=%d F=%d B=%d", d,
              num_features, batch);
    const int64_t P = (int64_t)num_features * (num_features - 1) / 2;
    CHECK_ARG(dout_ld >= d + P + padding && t_ld >= (int64_t)num_features * d && dx_ld >= d &&
                  dt_ld >= (int64_t)num_features * d,
              "dlrm_interact_bwd: leading dimensions too small");
    CHECK_ARG(batch == 0 || (dout && t && dx && dt), "dlrm_interact_bwd: null buffer");
    return launch_interact_bwd(ctx, dtype, d, num_features, batch, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld);
}

// ---- Implementation 2 pieces (interact.jl:176-215, :503-551)
int dlrm_triangular_slice(dlrm_ctx* ctx, int dtype, int sz, int batch, const void* z, int64_t z_batch_stride,
                          void* out, int64_t out_ld) {
    CHECK_ARG(ctx, "dlrm_triangular_slice: null ctx");
    CHECK_ARG(dtype == DLRM_F32 || dtype == DLRM_BF16, "dlrm_triangular_slice: dtype %d", dtype);
    CHECK_ARG(sz >= 1 && batch >= 0, "dlrm_triangular_slice: sz=%d batch=%d", sz, batch);
    CHECK_ARG(z_batch_stride >= (int64_t)sz * sz && out_ld >= (int64_t)sz * (sz - 1) / 2,
              "dlrm_triangular_slice: strides too small");
    CHECK_ARG(batch == 0 || sz < 2 || (z && out), "dlrm_triangular_slice: null buffer");  // sz = 1: no pairs
    return launch_triangular_slice(ctx, dtype, sz, batch, z, z_batch_stride, out, out_ld);
}

int dlrm_triangular_slice_back(dlrm_ctx* ctx, int dtype, int sz, int batch, const void* dy, int64_t dy_ld, void* a,
                               int64_t a_batch_stride, int symmetric) {
    CHECK_ARG(ctx, "dlrm_triangular_slice_back: null ctx");
    CHECK_ARG(dtype == DLRM_F32 || dtype == DLRM_BF16, "dlrm_triangular_slice_back: dtype %d", dtype);
    CHECK_ARG(sz >= 1 && batch >= 0, "dlrm_triangular_slice_back: sz=%d batch=%d", sz, batch);
    CHECK_ARG(a_batch_stride >= (int64_t)sz * sz && dy_ld >= (int64_t)sz * (sz - 1) / 2,
              "dlrm_triangular_slice_back: strides too small");
    CHECK_ARG(batch == 0 || (a && (sz < 2 || dy)), "dlrm_triangular_slice_back: null buffer");
    return launch_triangular_slice_back(ctx, dtype, sz, batch, dy, dy_ld, a, a_batch_stride, symmetric ? 1 : 0);
}

int dlrm_self_batched_mul(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch, const void* t, int64_t t_ld,
                          void* z, int64_t z_batch_stride) {
    CHECK_ARG(ctx, "dlrm_self_batched_mul: null ctx");
    CHECK_ARG(dtype == DLRM_F32 || dtype == DLRM_BF16, "dlrm_self_batched_mul: dtype %d", dtype);
    CHECK_ARG(d > 0 && num_features >= 1 && batch >= 0, "dlrm_self_batched_mul: d=%d F=%d B=%d", d, num_features, batch);
    if (num_features > 90) return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "dlrm_self_batched_mul: F=%d > 90", num_features);
    CHECK_ARG(t_ld >= (int64_t)num_features * d && z_batch_stride >= (int64_t)num_features * num_features,
              "dlrm_self_batched_mul: strides too small");
    CHECK_ARG(batch == 0 || (t && z), "dlrm_self_batched_mul: null buffer");
    return launch_self_batched_mul(ctx, dtype, d, num_features, batch, t, t_ld, z, z_batch_stride);
}

int dlrm_self_batched_mul_back(dlrm_ctx* ctx, int dtype, int d, int num_features, int batch, const void* t,
                               int64_t t_ld, const void* dz, int64_t dz_batch_stride, float* dt, int64_t dt_ld) {
    CHECK_ARG(ctx, "dlrm_self_batched_mul_back: null ctx");
    CHECK_ARG(dtype == DLRM_F32 || dtype == DLRM_BF16, "dlrm_self_batched_mul_back: dtype %d", dtype);
    CHECK_ARG(d > 0 && num_features >= 1 && batch >= 0, "dlrm_self_batched_mul_back: d=%d F=%d B=%d", d, num_features,
              batch);
    if (num_features > 90)
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "dlrm_self_batched_mul_back: F=%d > 90", num_features);
    CHECK_ARG(t_ld >= (int64_t)num_features * d && dz_batch_stride >= (int64_t)num_features * num_features &&
                  dt_ld >= (int64_t)num_features * d,
              "dlrm_self_batched_mul_back: strides too small");
    CHECK_ARG(batch == 0 || (t && dz && dt), "dlrm_self_batched_mul_back: null buffer");
    return launch_self_batched_mul_back(ctx, dtype, d, num_features, batch, t, t_ld, dz, dz_batch_stride, dt, dt_ld);
}

int dlrm_interact_bwd_gather(dlrm_ctx* ctx, const dlrm_tables* tb, dlrm_indexer* ix, const void* indices, int itype,
                             int64_t table_stride, int index_base, int batch, int lookups, const void* x,
                             int64_t x_ld, const void* dout, int64_t dout_ld, int padding, float* dx, int64_t dx_ld,
                             float* dt, int64_t dt_ld) {
    CHECK_ARG(ctx && tb, "dlrm_interact_bwd_gather: null ctx/tables");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, lookups);
    if (rc) return rc;
    CHECK_ARG(lookups == 1, "dlrm_interact_bwd_gather: one-hot lookups only (L=%d: use dlrm_interact_bwd on ys)",
              lookups);
    const int d = tb->D, F = tb->T + 1;
    const int64_t P = (int64_t)F * (F - 1) / 2;
    CHECK_ARG(padding >= 0 && x_ld >= d && dout_ld >= d + P + padding && dx_ld >= d && dt_ld >= (int64_t)F * d,
              "dlrm_interact_bwd_gather: leading dimensions too small");
    CHECK_ARG(batch == 0 || (x && dout && dx && dt), "dlrm_interact_bwd_gather: null buffer");
    if (ix) {
        CHECK_ARG(tb->T == ix->T, "dlrm_interact_bwd_gather: indexer has %d tables, tables has %d", ix->T, tb->T);
        CHECK_ARG((int64_t)batch * lookups <= ix->dev.cap,
                  "dlrm_interact_bwd_gather: batch*lookups %lld > indexer capacity %lld", (long long)batch * lookups,
                  (long long)ix->dev.cap);
    }
    if (ix) ix->dev.vshift = 0;
    rc = launch_interact_bwd_gather(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype, table_stride,
                                    index_base, lookups, d, batch, x, x_ld, dout, dout_ld, dx, dx_ld, dt, dt_ld,
                                    ix ? &ix->dev : nullptr, tb->h_desc.data());
    if (rc || !ix) return rc;
    // as dlrm_indexer_build: a following update may pass DLRM_UPDATE_PREBUILT
    record_build(ix, false, indices, itype, table_stride, index_base, batch, lookups);
    return DLRM_OK;
}

int dlrm_interact_bwd_blocked(dlrm_ctx* ctx, const dlrm_tables* tb, const void* indices, int itype,
                              int64_t table_stride, int index_base, int batch, const void* x, int64_t x_ld,
                              const void* dout, int64_t dout_ld, int padding, float* dx, int64_t dx_ld, float* dst,
                              const int64_t* dst_base, const int64_t* dst_ld) {
    CHECK_ARG(ctx && tb, "dlrm_interact_bwd_blocked: null ctx/tables");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, 1);
    if (rc) return rc;
    const int d = tb->D, F = tb->T + 1;
    const int64_t P = (int64_t)F * (F - 1) / 2;
    CHECK_ARG(padding >= 0 && x_ld >= d && dout_ld >= d + P + padding && dx_ld >= d,
              "dlrm_interact_bwd_blocked: leading dimensions too small");
    CHECK_ARG(batch == 0 || tb->T == 0 || (x && dout && dx && dst && dst_base && dst_ld),
              "dlrm_interact_bwd_blocked: null buffer");
    return launch_interact_bwd_blocked(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype, table_stride,
                                       index_base, 1, d, batch, x, x_ld, dout, dout_ld, dx, dx_ld, dst, dst_base,
                                       dst_ld, tb->h_desc.data());
}

// --------------------------------------------------------------------------- indexer
// Footprint.  The per-part arrays (perm, seg_start, seg_row, chunks, hot, hot_slice, hot_cnt: 92 B
// per slot; + 20 B of HBM sort scratch above 2048 positions) are cap slots per table: the wave
// builds pack a table's parts back to back (common.hpp kSegPad, "compact" layout), whatever the
// parts (256 per table at 32768 positions).  Only the in-LDS parts build of 4096 < N <= 8192
// (fast_index_table, 8 parts, v * cap) needs 8 virtual tables of cap slots per table, so an
// indexer whose cap is in that range is carved with 8.  (Round 5 gave every wave-build part a whole
// cap and re-carved on first use: 128 x the table at 16384 positions, ~7 GB per indexer for 26
// tables)  Partial rows of multi-slice hot segments are per real table (the wave
// build's item map indexes them by its flat slice number, at most pcap per table), times the <= 8
// parts of the builds without an item map.
static int64_t partial_rows(const dlrm_indexer* ix) {
    const int64_t T0 = ix->T > 0 ? ix->T : 1;
    const int64_t cap = ix->dev.cap;
    const int np = cap <= kPartsMaxN ? 8 : 1;
    return T0 * np * ix->dev.pcap;
}

// Carves every array of the indexer for `parts` virtual tables per table (contents reset).
static int indexer_carve(dlrm_ctx* ctx, dlrm_indexer* ix, int parts) {
    const int64_t cap = ix->dev.cap;
    const int64_t T0 = ix->T > 0 ? ix->T : 1;
    const int64_t T = (int64_t)parts * T0;
    const int64_t hs = ix->dev.hsize;
    // the largest wave build this indexer takes: 2^vw parts per table, T0 << vw / 4 workgroups (>= 64
    // parts: the builds of <= 2048 positions may take 32 or 64, dlrm_indexer_set_parts)
    const int vw = std::max(wave_vshift(cap < kWaveMaxN ? cap : kWaveMaxN), 6);
    const int64_t TW = T0 << vw;
    // carve every array out of one allocation (16-B aligned pieces)
    struct Piece { void** p; size_t bytes; };
    const size_t n = (size_t)(T * cap), n0 = (size_t)(T0 * cap);
    const size_t n1 = (size_t)std::max(T * (cap + 1), T0 * (cap + kSegPad));  // (compact: a sentinel per part)
    const size_t ncnt = (size_t)std::max(T, TW);
    // the wave build's flat item lists: kResLists sub-lists of res_stride records (indexer.hpp); the
    // HBM sort scratch (5 arrays, compact) for the builds of more than 2048 positions
    const size_t nrec = (size_t)kResLists * (size_t)res_stride((int)(TW / 4), cap, vw) + 64;
    const int64_t wstride = cap > kStepIndexMaxN ? T0 * cap + 64 : 0;
    IndexerDev d = ix->dev;
    float* partial_keep = ix->partial_big ? d.partial : nullptr;  // (a grown partial buffer stays)
    Piece pieces[] = {
        {(void**)&d.keys0, n0 * 4},    {(void**)&d.keys1, n0 * 4},  {(void**)&d.vals0, n0 * 4},
        {(void**)&d.vals1, n0 * 4},    {(void**)&d.perm, n * 4},    {(void**)&d.seg_start, n1 * 4},
        {(void**)&d.seg_row, n * 4},   {(void**)&d.chunks, n * 32}, {(void**)&d.hot, n * 16},
        {(void**)&d.hot_slice, n * 16}, {(void**)&d.hot_cnt, n * 4},
        {(void**)&d.partial, partial_keep ? 0 : (size_t)partial_rows(ix) * kPartialDim * 4},
        {(void**)&d.counts, ncnt * 32},   {(void**)&d.single, n0},
        {(void**)&ix->prep_err, 16},
        {(void**)&d.slice_rec, nrec * 32}, {(void**)&d.chunk_rec, nrec * 32},
        {(void**)&d.wscratch, (size_t)wstride * 5 * 4},
        {(void**)&d.item_tot, 64},     {(void**)&d.build_arrive, 2048},
        // hash indexer arrays (only when a build can exceed the in-LDS indexer's kFastMaxN)
        {(void**)&d.pslot, hs ? n0 * 4 : 0},   {(void**)&d.hent, (size_t)(T0 * hs) * 8},
        {(void**)&d.hseg, (size_t)(T0 * hs) * 8},
        {(void**)&d.hfill, (size_t)(T0 * hs) * 4}, {(void**)&d.hstate, hs ? (size_t)T0 * 32 : 0},
    };
    size_t total = 0;
    for (auto& pc : pieces) total += (pc.bytes + 255) & ~(size_t)255;
    int rc = hip_set(ctx);
    void* block = nullptr;
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipMalloc(&block, total), "hipMalloc(indexer)");
    if (rc == DLRM_OK) rc = ctx_hip(ctx, hipMemset(block, 0, total), "hipMemset(indexer)");
    char* base = (char*)block;
    if (rc == DLRM_OK)
        for (auto& pc : pieces) {
            *pc.p = pc.bytes ? base : nullptr;
            base += (pc.bytes + 255) & ~(size_t)255;
        }
    if (rc == DLRM_OK && hs)  // every slot starts empty (the alloc pass resets the slots it used)
        rc = ctx_hip(ctx, hipMemset(d.hent, 0xff, (size_t)(T0 * hs) * 8), "hipMemset(hash slots)");
    if (rc != DLRM_OK) {
        if (block) (void)hipFree(block);
        return rc;
    }
    if (partial_keep) d.partial = partial_keep;
    d.wstride = wstride;
    if (ix->block) {  // (nothing in flight may still read the old arrays)
        (void)hipDeviceSynchronize();
        (void)hipFree(ix->block);
    }
    ix->block = block;
    ix->dev = d;
    ix->TV = (int)T;
    ix->bytes = total;
    ix->built = ix->prepared = ix->singles_done = false;
    ix->dev.has_map = 0;
    ix->dev.build_err = nullptr;
    return DLRM_OK;
}

// Whether a wave build of `batch` positions per table fits this indexer (compact layout: any parts;
// the flat records hold global perm entries in int32).
static bool wave_fits(const dlrm_indexer* ix, int64_t batch) {
    return batch <= ix->dev.cap && batch <= kWaveMaxN && (int64_t)(ix->T > 0 ? ix->T : 1) * ix->dev.cap < (1ll << 31);
}

int dlrm_indexer_create(dlrm_ctx* ctx, int num_tables, int64_t max_lookups, dlrm_indexer** out) {
    CHECK_ARG(ctx && out, "dlrm_indexer_create: null argument");
    *out = nullptr;
    CHECK_ARG(num_tables >= 0 && max_lookups >= 0 && max_lookups < (1ll << 31), "dlrm_indexer_create: T=%d cap=%lld",
              num_tables, (long long)max_lookups);
    dlrm_indexer* ix = new (std::nothrow) dlrm_indexer();
    if (!ix) return DLRM_E_NOMEM;
    ix->ctx = ctx;
    ix->T = num_tables;
    const int64_t cap = max_lookups > 0 ? max_lookups : 1;
    ix->dev.cap = cap;
    ix->dev.pcap = indexer_slice_cap(cap);
    ix->dev.pdim = kPartialDim;
    ix->dev.chunk_max = kChunk;
    const int64_t hs = cap > kFastMaxN ? hix_table_slots(cap) : 0;
    ix->dev.hsize = hs;
    ix->dev.hbits = 0;
    while (((int64_t)1 << ix->dev.hbits) < hs) ++ix->dev.hbits;
    // 8 virtual tables per table for the in-LDS parts build of kFastMaxN < N <= kPartsMaxN (fast_index_table;
    // build_vshift <= 3), else one: every wave build packs its parts per table
    const int parts = cap > kFastMaxN && cap <= kPartsMaxN ? (1 << 3) : 1;
    const int rc = indexer_carve(ctx, ix, parts);
    if (rc != DLRM_OK) {
        delete ix;
        return rc;
    }
    *out = ix;
    return DLRM_OK;
}

int dlrm_indexer_set_chunk(dlrm_ctx* ctx, dlrm_indexer* ix, int max_positions) {
    CHECK_ARG(ctx && ix, "dlrm_indexer_set_chunk: null argument");
    CHECK_ARG(max_positions == 16 || max_positions == 32, "dlrm_indexer_set_chunk: %d (16 or 32)", max_positions);
    ix->dev.chunk_max = max_positions;
    return DLRM_OK;
}

int dlrm_indexer_set_parts(dlrm_ctx* ctx, dlrm_indexer* ix, int parts) {
    CHECK_ARG(ctx && ix, "dlrm_indexer_set_parts: null argument");
    CHECK_ARG(parts == 0 || parts == 16 || parts == 32 || parts == 64, "dlrm_indexer_set_parts: %d (0, 16, 32 or 64)",
              parts);
    ix->parts_log2 = parts == 64 ? 6 : (parts == 32 ? 5 : (parts == 16 ? 4 : 0));
    return DLRM_OK;
}

int dlrm_indexer_reserve(dlrm_ctx* ctx, dlrm_indexer* ix, int batch) {
    CHECK_ARG(ctx && ix, "dlrm_indexer_reserve: null argument");
    CHECK_ARG(batch >= 0 && batch <= ix->dev.cap, "dlrm_indexer_reserve: batch %d > capacity %lld", batch,
              (long long)ix->dev.cap);
    // (round 6: the wave builds' compact layout needs no re-carving; nothing to do)
    return DLRM_OK;
}

int dlrm_indexer_bytes(const dlrm_indexer* ix, int64_t* bytes) {
    if (!ix || !bytes) return DLRM_E_ARG;
    *bytes = (int64_t)ix->bytes + (ix->partial_big ? partial_rows(ix) * (int64_t)ix->dev.pdim * 4 : 0);
    return DLRM_OK;
}

int dlrm_indexer_destroy(dlrm_indexer* ix) {
    if (!ix) return DLRM_OK;
    if (ix->block) (void)hipFree(ix->block);
    if (ix->partial_big) (void)hipFree(ix->partial_big);
    delete ix;
    return DLRM_OK;
}

// vshift of a standalone split build of N positions per table: the parts build where it applies
static int build_vshift(const dlrm_indexer* ix, int64_t N, bool split) {
    const int p = knobs().build_parts ? knobs().build_parts : (1 << kPartsLog2);
    const int lg = p >= 8 ? 3 : (p >= 4 ? 2 : 1);
    return split && N > kFastMaxN && N <= kPartsMaxN && has_parts(ix, lg) ? lg : 0;
}

int dlrm_indexer_build(dlrm_ctx* ctx, dlrm_indexer* ix, const dlrm_tables* tb, const void* indices, int itype,
                       int64_t table_stride, int index_base, int batch, int lookups) {
    CHECK_ARG(ctx && ix && tb, "dlrm_indexer_build: null argument");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, lookups);
    if (rc) return rc;
    CHECK_ARG(tb->T == ix->T, "dlrm_indexer_build: indexer has %d tables, tables has %d", ix->T, tb->T);
    CHECK_ARG((int64_t)batch * lookups <= ix->dev.cap, "dlrm_indexer_build: batch*lookups %lld > capacity %lld",
              (long long)batch * lookups, (long long)ix->dev.cap);
    // the split form where the builds support it: once-hit positions flagged (single[]) instead of
    // listed as one-position chunks; the apply then updates them with no descriptor read
    const int64_t N = (int64_t)batch * lookups;
    const bool split = N <= kFastMaxN || (ix->dev.hsize && N <= kHixMaxN);
    if (split && N > kPartsMaxN && wave_fits(ix, N) && !knobs().bag_hash) {
        // pooled bags (configs[4]: 20480 positions per table) and other large batches: the bag build
        // (update.hip: count, place by part, then the wave build's per-part sort; 2^wave_vshift(N)
        // parts per table, flat item map) instead of the hash build (4 launches, global atomics;
        // round 5: 146 us and 13x its algorithmic bytes for configs[4]).  It groups positions
        // p = b L + k; the apply maps p to its bag.  Bounds errors go to the ctx's flag, as every
        // dlrm_indexer_build's.
        ix->built = false;
        // half the parts of the wave builds (128 to 256 positions per part; configs[4] at 20480: 128
        // parts, 50.6 us against 66.7 us with 256 -- half the sort workgroups, each still sorting in
        // registers)
        ix->dev.vshift = knobs().bag_vs >= 2 && knobs().bag_vs <= wave_vshift(ix->dev.cap < kWaveMaxN ? ix->dev.cap : kWaveMaxN)
                             ? knobs().bag_vs : wave_vshift(N) - 1;
        rc = launch_bag_build(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride, index_base, (int)N,
                              ctx_error_word(ctx));
        if (rc) return rc;
        record_build(ix, true, indices, itype, table_stride, index_base, batch, lookups);
        ix->dev.has_map = 1;
        return DLRM_OK;
    }
    ix->dev.vshift = build_vshift(ix, N, split);
    rc = launch_indexer_build(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride, index_base, batch, lookups,
                              split);
    if (rc) return rc;
    record_build(ix, split, indices, itype, table_stride, index_base, batch, lookups);
    return DLRM_OK;
}

int dlrm_indexer_build_split(dlrm_ctx* ctx, dlrm_indexer* ix, const dlrm_tables* tb, const void* indices, int itype,
                             int64_t table_stride, int index_base, int batch) {
    CHECK_ARG(ctx && ix && tb, "dlrm_indexer_build_split: null argument");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, 1);
    if (rc) return rc;
    CHECK_ARG(tb->T == ix->T, "dlrm_indexer_build_split: indexer has %d tables, tables has %d", ix->T, tb->T);
    CHECK_ARG(batch <= ix->dev.cap, "dlrm_indexer_build_split: batch %d > capacity %lld", batch,
              (long long)ix->dev.cap);
    ix->built = false;
    // above the in-LDS build's 4096 positions: the bag build (configs[2]'s next-batch build at 8192, on
    // a side stream beside the step: 94.5 vs 96.4 us per step with the in-LDS parts build -- its
    // three launches are slower alone, 38.7 vs 17.7 us, but their small workgroups run beside the
    // step's kernels, where the parts build's 104 workgroups of 136 KB LDS each held a whole CU;
    // DESIGN.md §3 round 6).  DLRM_BAG_SPLIT=0: the parts / hash builds.
    if (knobs().bag_split && batch > kFastMaxN && wave_fits(ix, batch)) {
        ix->dev.vshift = wave_vshift(batch) - 1;
        rc = launch_bag_build(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride, index_base, batch,
                              ctx_error_word(ctx));
        if (rc) return rc;
        record_build(ix, true, indices, itype, table_stride, index_base, batch, 1);
        ix->dev.has_map = 1;
        return DLRM_OK;
    }
    ix->dev.vshift = build_vshift(ix, batch, true);
    rc = launch_indexer_build(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride, index_base, batch, 1,
                              true, nullptr);
    if (rc) return rc;
    record_build(ix, true, indices, itype, table_stride, index_base, batch, 1);
    return DLRM_OK;
}

int dlrm_indexer_prepare(dlrm_ctx* ctx, dlrm_indexer* ix, const dlrm_tables* tb, const void* indices, int itype,
                         int64_t table_stride, int index_base, int batch) {
    CHECK_ARG(ctx && ix && tb, "dlrm_indexer_prepare: null argument");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, 1);
    if (rc) return rc;
    CHECK_ARG(tb->T == ix->T, "dlrm_indexer_prepare: indexer has %d tables, tables has %d", ix->T, tb->T);
    CHECK_ARG(batch <= ix->dev.cap, "dlrm_indexer_prepare: batch %d > capacity %lld", batch, (long long)ix->dev.cap);
    const int vs = wave_parts_log2(batch, ix);
    if (!wave_fits(ix, batch))
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "dlrm_indexer_prepare: batch %d (the wave build: batch <= %d, "
                        "tables x capacity < 2^31)", batch, kWaveMaxN);
    ix->built = false;
    ix->prepared = false;
    ix->dev.vshift = vs;
    // bounds errors go to the indexer's own word, not the ctx's flag: this build usually runs on a
    // side stream beside the current step, whose kernels read the ctx's flag to decide whether to
    // write their rows.  The next forward / lookup of these indices raises them on the ctx's flag;
    // the apply of this indexer folds the word in as well (a prebuilt update without a lookup).
    rc = ctx_hip(ctx, hipMemsetAsync(ix->prep_err, 0, sizeof(unsigned), ctx->stream), "clear build bounds word");
    if (rc) return rc;
    rc = launch_step_prepare(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride, index_base, batch,
                             ix->prep_err);
    if (rc) return rc;
    record_build(ix, true, indices, itype, table_stride, index_base, batch, 1);
    ix->prepared = true;
    ix->dev.has_map = 1;
    ix->dev.build_err = ix->prep_err;
    return DLRM_OK;
}

// One (virtual) table's build, whole: rows, grouped positions, segment starts.
struct IndexerTable {
    std::vector<uint32_t> rows;
    std::vector<int32_t> perm, seg_start;
};
static int read_indexer_table(dlrm_ctx* ctx, const dlrm_indexer* ix, int v, IndexerTable& o) {
    int32_t cnt[8];
    int rc = ctx_hip(ctx, hipMemcpy(cnt, ix->dev.counts + (int64_t)v * 8, sizeof(cnt), hipMemcpyDeviceToHost), "read");
    if (rc) return rc;
    const int64_t U = cnt[0], NV = cnt[4];
    // (a wave build's parts are packed per table: IndexerDev::part_off / seg_off)
    const int vs = ix->dev.vshift;
    const int64_t cap = ix->dev.cap;
    const int64_t off = ix->dev.has_map ? (int64_t)(v >> vs) * cap + cnt[kCntOff] : (int64_t)v * cap;
    const int64_t soff = ix->dev.has_map ? (int64_t)(v >> vs) * (cap + kSegPad) + cnt[kCntOff] + (v & ((1 << vs) - 1))
                                         : (int64_t)v * (cap + 1);
    o.rows.resize(U);
    o.perm.resize(NV);
    o.seg_start.resize(U + 1);
    if (U) rc = ctx_hip(ctx, hipMemcpy(o.rows.data(), ix->dev.seg_row + off, U * 4, hipMemcpyDeviceToHost), "read");
    if (rc == DLRM_OK && NV)
        rc = ctx_hip(ctx, hipMemcpy(o.perm.data(), ix->dev.perm + off, NV * 4, hipMemcpyDeviceToHost), "read");
    if (rc == DLRM_OK)
        rc = ctx_hip(ctx, hipMemcpy(o.seg_start.data(), ix->dev.seg_start + soff,
                                    (U + 1) * 4, hipMemcpyDeviceToHost), "read");
    return rc;
}

int dlrm_indexer_state(const dlrm_indexer* ix, unsigned* state) {
    if (!ix || !state) return DLRM_E_ARG;
    *state = (ix->built ? DLRM_IX_BUILT : 0u) | (ix->split ? DLRM_IX_SPLIT : 0u) |
             (ix->prepared ? DLRM_IX_PREPARED : 0u) | (ix->singles_done ? DLRM_IX_SINGLES_DONE : 0u);
    return DLRM_OK;
}

int dlrm_indexer_read(dlrm_ctx* ctx, const dlrm_indexer* ix, int table, int64_t* num_unique, int64_t* rows,
                      int64_t* positions, int64_t* seg_start, int64_t cap) {
    CHECK_ARG(ctx && ix && num_unique, "dlrm_indexer_read: null argument");
    CHECK_ARG(ix->built, "dlrm_indexer_read: indexer not built");
    CHECK_ARG(table >= 0 && table < ix->T, "dlrm_indexer_read: table %d", table);
    int rc = ctx_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if (rc) return rc;
    IndexerTable tt;
    if (ix->dev.vshift == 0) {
        rc = read_indexer_table(ctx, ix, table, tt);
    } else {
        // a forward-launch build: merge the table's parts (each sorted by row)
        const int np = 1 << ix->dev.vshift;
        std::vector<IndexerTable> h(np);
        for (int q = 0; q < np && rc == DLRM_OK; ++q) rc = read_indexer_table(ctx, ix, table * np + q, h[q]);
        std::vector<size_t> k(np, 0);
        tt.seg_start.assign(1, 0);
        for (;;) {
            int e = -1;
            for (int q = 0; q < np && rc == DLRM_OK; ++q)
                if (k[q] < h[q].rows.size() && (e < 0 || h[q].rows[k[q]] < h[e].rows[k[e]])) e = q;
            if (e < 0) break;
            const size_t u = k[e]++;
            tt.rows.push_back(h[e].rows[u]);
            for (int32_t i = h[e].seg_start[u]; i < h[e].seg_start[u + 1]; ++i) tt.perm.push_back(h[e].perm[i]);
            tt.seg_start.push_back((int32_t)tt.perm.size());
        }
    }
    if (rc) return rc;
    const int64_t U = (int64_t)tt.rows.size(), NV = (int64_t)tt.perm.size();
    *num_unique = U;
    if (rows)
        for (int64_t i = 0; i < U && i < cap; ++i) rows[i] = tt.rows[i];
    if (positions && seg_start) {
        for (int64_t i = 0; i < NV && i < cap; ++i) positions[i] = tt.perm[i];
        for (int64_t i = 0; i <= U && i <= cap; ++i) seg_start[i] = tt.seg_start[i];
    }
    return DLRM_OK;
}

// multi-slice hot segments keep partial rows of D elements (allocated on first use for D > kPartialDim;
// not on a launch path that is captured: the first update of a shape runs before capture)
static int ensure_partials(dlrm_ctx* ctx, dlrm_indexer* ix, int D) {
    if (D <= ix->dev.pdim) return DLRM_OK;
    void* p = nullptr;
    int rc = hip_set(ctx);
    if (rc == DLRM_OK)
        rc = ctx_hip(ctx, hipMalloc(&p, (size_t)partial_rows(ix) * D * 4), "hipMalloc(indexer partials)");
    if (rc) return rc;
    if (ix->partial_big) (void)hipFree(ix->partial_big);
    ix->partial_big = p;
    ix->dev.partial = (float*)p;
    ix->dev.pdim = D;
    return DLRM_OK;
}

int dlrm_sgd_update(dlrm_ctx* ctx, dlrm_tables* tb, dlrm_indexer* ix, unsigned flags, const void* indices, int itype,
                    int64_t table_stride, int index_base, int batch, int lookups, const void* grad, int grad_dtype,
                    int64_t grad_ld, int64_t grad_offset, float lr) {
    CHECK_ARG(ctx && tb, "dlrm_sgd_update: null ctx/tables");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, lookups);
    if (rc) return rc;
    CHECK_ARG(grad_dtype == DLRM_F32 || grad_dtype == DLRM_BF16, "dlrm_sgd_update: grad dtype %d", grad_dtype);
    CHECK_ARG(grad_offset >= 0 && grad_ld >= grad_offset + (int64_t)tb->T * tb->D, "dlrm_sgd_update: grad_ld too small");
    CHECK_ARG(batch == 0 || tb->T == 0 || grad, "dlrm_sgd_update: null grad");
    if (flags & DLRM_UPDATE_ATOMIC) {
        if (tb->dtype != DLRM_F32)
            return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "dlrm_sgd_update: atomic mode needs fp32 tables");
        return launch_sgd_atomic(ctx, tb->d_desc, tb->T, tb->D, indices, itype, table_stride, index_base, batch,
                                 lookups, grad, grad_dtype, grad_ld, grad_offset, lr);
    }
    CHECK_ARG(ix, "dlrm_sgd_update: deterministic mode needs an indexer");
    if (flags & DLRM_UPDATE_PREBUILT) {
        if (!built_from(ix, indices, itype, table_stride, index_base, batch, lookups))
            return ctx_fail(ctx, DLRM_E_STATE, "dlrm_sgd_update: indexer was not built from these indices");
    } else {
        rc = dlrm_indexer_build(ctx, ix, tb, indices, itype, table_stride, index_base, batch, lookups);
        if (rc) return rc;
    }
    rc = ensure_partials(ctx, ix, tb->D);
    if (rc) return rc;
    // a split indexer (dlrm_indexer_build's default form, or dlrm_step_fwd's): its once-hit
    // positions are this launch's too -- unless a split backward (dlrm_step_bwd) has updated them
    // already, in which case only the repeated rows are left (their dt rows are all it wrote)
    const SinglesArgs sa{(ix->split && !ix->singles_done) ? ix->dev.single : nullptr, indices, itype, table_stride,
                         index_base, batch * lookups};
    return launch_sgd_apply(ctx, ix->dev, tb->d_desc, tb->aligned16, tb->T, tb->D, tb->dtype, lookups,
                            (int64_t)batch * lookups, grad, grad_dtype, grad_ld, grad_offset, lr, sa);
}

// ----------------------------------------------------------------------- training step
int dlrm_step_fwd(dlrm_ctx* ctx, const dlrm_tables* tb, dlrm_indexer* ix, const void* indices, int itype,
                  int64_t table_stride, int index_base, int batch, const void* x, int64_t x_ld, void* out,
                  int64_t out_ld, int padding) {
    CHECK_ARG(ctx && tb && ix, "dlrm_step_fwd: null ctx/tables/indexer");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, 1);
    if (rc) return rc;
    CHECK_ARG(tb->T == ix->T, "dlrm_step_fwd: indexer has %d tables, tables has %d", ix->T, tb->T);
    CHECK_ARG(batch <= ix->dev.cap, "dlrm_step_fwd: batch %d > indexer capacity %lld", batch, (long long)ix->dev.cap);
    const int d = tb->D, F = tb->T + 1;
    const int64_t P = (int64_t)F * (F - 1) / 2;
    CHECK_ARG(padding >= 0 && x_ld >= d && out_ld >= d + P + padding, "dlrm_step_fwd: leading dimensions too small");
    CHECK_ARG(batch == 0 || (x && out), "dlrm_step_fwd: null buffer");
    if (ix->prepared && built_from(ix, indices, itype, table_stride, index_base, batch, 1)) {
        // built by the previous step's apply launch (dlrm_step_bwd_prepare): the gather alone
        ix->prepared = false;
        rc = launch_lookup_interact_fwd(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype, table_stride,
                                        index_base, 1, d, batch, x, x_ld, nullptr, 0, out, out_ld, padding, tb->h_desc.data());
        if (rc != DLRM_E_UNSUPPORTED) return rc;  // (no fused forward for this x: build below)
    }
    ix->prepared = false;
    ix->built = false;
    // the wave build in the forward's launch (vshift >= 2: it also writes the apply's item map)
    ix->dev.vshift = ix->dev.cap <= kWaveApplyMaxN && wave_fits(ix, batch) ? wave_parts_log2(kStepIndexMaxN, ix) : 0;
    rc = launch_step_fwd(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype, table_stride, index_base, d,
                         batch, x, x_ld, out, out_ld, padding, ix->dev, tb->h_desc.data());
    if (rc == DLRM_OK) {
        record_build(ix, true, indices, itype, table_stride, index_base, batch, 1);
        ix->dev.has_map = ix->dev.vshift >= 2 ? 1 : 0;
        return DLRM_OK;
    }
    if (rc != DLRM_E_UNSUPPORTED) return rc;
    ix->dev.vshift = 0;
    const bool split_ok = step_split_supported(tb->aligned16, tb->T, tb->dtype, d, x, x_ld);
    if (split_ok && batch <= kFastMaxN) {
        // no single-launch form for this shape (B > 2048): the fused forward, then the split
        // indexer in LDS (one 1024-thread workgroup per table)
        rc = launch_lookup_interact_fwd(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype,
                                        table_stride, index_base, 1, d, batch, x, x_ld, nullptr, 0, out, out_ld,
                                        padding, tb->h_desc.data());
        if (rc == DLRM_OK)
            rc = launch_indexer_build(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride, index_base,
                                      batch, 1, true, nullptr);
        if (rc == DLRM_OK) {
            record_build(ix, true, indices, itype, table_stride, index_base, batch, 1);
            return DLRM_OK;
        }
        if (rc != DLRM_E_UNSUPPORTED) return rc;
    }
    const int pvs = build_vshift(ix, batch, true);
    if (split_ok && (pvs > 0 || ix->dev.hsize) && batch > kFastMaxN && batch <= kHixMaxN) {
        // large batch: the split build (once-hit rows left to dlrm_step_bwd) -- in LDS by table
        // parts up to kPartsMaxN, else the hash build -- on the side stream beside the fused
        // forward (launched below); the main stream joins it
        rc = ensure_side(ctx);
        if (rc) return rc;
        rc = ctx_hip(ctx, hipEventRecord(ctx->ev_fork, ctx->stream), "hipEventRecord(fork)");
        if (rc == DLRM_OK) rc = ctx_hip(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0), "hipStreamWaitEvent(side)");
        ix->dev.vshift = pvs;
        if (rc == DLRM_OK)
            rc = pvs > 0 ? launch_indexer_build(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride,
                                                index_base, batch, 1, true, ctx->side)
                         : launch_hix_build(ctx, ix->dev, tb->d_desc, tb->T, indices, itype, table_stride, index_base,
                                            batch, true, ctx->side);
        if (rc == DLRM_OK) rc = ctx_hip(ctx, hipEventRecord(ctx->ev_join, ctx->side), "hipEventRecord(join)");
        if (rc) return rc;
        rc = launch_lookup_interact_fwd(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype,
                                        table_stride, index_base, 1, d, batch, x, x_ld, nullptr, 0, out, out_ld,
                                        padding, tb->h_desc.data());
        const int rj = ctx_hip(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0), "hipStreamWaitEvent(main)");
        if (rc == DLRM_E_UNSUPPORTED)
            return ctx_fail(ctx, DLRM_E_UNSUPPORTED,
                            "dlrm_step_fwd: no fused forward for this shape (16-B aligned rows and x, F <= 96 needed)");
        if (rc || rj) return rc ? rc : rj;
        record_build(ix, true, indices, itype, table_stride, index_base, batch, 1);
        return DLRM_OK;
    }
    // no single-launch form for this shape: the fused forward, then the (unsplit) indexer
    rc = launch_lookup_interact_fwd(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype, table_stride,
                                    index_base, 1, d, batch, x, x_ld, nullptr, 0, out, out_ld, padding, tb->h_desc.data());
    if (rc == DLRM_E_UNSUPPORTED)
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED,
                        "dlrm_step_fwd: no fused forward for this shape (16-B aligned rows and x, F <= 96 needed)");
    if (rc) return rc;
    return dlrm_indexer_build(ctx, ix, tb, indices, itype, table_stride, index_base, batch, 1);
}

static int step_bwd_impl(dlrm_ctx* ctx, dlrm_tables* tb, dlrm_indexer* ix, const void* indices, int itype,
                         int64_t table_stride, int index_base, int batch, const void* x, int64_t x_ld,
                         const void* dout, int64_t dout_ld, int padding, float* dx, int64_t dx_ld, float* dt,
                         int64_t dt_ld, float lr, unsigned flags, const PrepArgs* prep) {
    CHECK_ARG(ctx && tb && ix, "dlrm_step_bwd: null ctx/tables/indexer");
    int rc = check_indices(ctx, tb, indices, itype, table_stride, batch, 1);
    if (rc) return rc;
    const int d = tb->D, F = tb->T + 1;
    const int64_t P = (int64_t)F * (F - 1) / 2;
    CHECK_ARG(padding >= 0 && x_ld >= d && dout_ld >= d + P + padding && dx_ld >= d && dt_ld >= (int64_t)F * d,
              "dlrm_step_bwd: leading dimensions too small");
    CHECK_ARG(batch == 0 || (x && dout && dx && dt), "dlrm_step_bwd: null buffer");
    if (!built_from(ix, indices, itype, table_stride, index_base, batch, 1))
        return ctx_fail(ctx, DLRM_E_STATE, "dlrm_step_bwd: the indexer was not built by dlrm_step_fwd from these indices");
    CHECK_ARG(flags != (DLRM_STEP_BWD_ONLY | DLRM_STEP_APPLY_ONLY), "dlrm_step_bwd: flags %u", flags);
    rc = ensure_partials(ctx, ix, tb->D);
    if (rc) return rc;
    // the split backward (once-hit rows updated there) where the shape has it; otherwise the
    // gather backward writes every dt row and the apply takes a split indexer's once-hit rows too
    const bool split_bwd = ix->split && step_split_supported(tb->aligned16, tb->T, tb->dtype, d, x, x_ld);
    if (flags & DLRM_STEP_APPLY_ONLY) {
        // the apply of a split build only completes a backward that stepped the once-hit rows
        if (split_bwd && !ix->singles_done)
            return ctx_fail(ctx, DLRM_E_STATE, "dlrm_step_bwd(APPLY_ONLY): no backward has run on this build");
        rc = DLRM_OK;
    } else if (split_bwd) {
        // a second backward on one build would step its once-hit rows twice
        if (ix->singles_done)
            return ctx_fail(ctx, DLRM_E_STATE,
                            "dlrm_step_bwd: this build's once-hit rows were already stepped (one backward per "
                            "dlrm_step_fwd)");
        CHECK_ARG((uintptr_t)dx % 16 == 0 && (uintptr_t)dt % 16 == 0 && dx_ld % 4 == 0 && dt_ld % 4 == 0,
                  "dlrm_step_bwd: dx and dt must be 16-B aligned with leading dimensions divisible by 4");
        rc = launch_step_bwd(ctx, tb->d_desc, tb->T, tb->dtype, indices, itype, table_stride, index_base, d, batch, x,
                             x_ld, dout, dout_ld, dx, dx_ld, dt, dt_ld, ix->dev, lr, tb->h_desc.data());
        if (rc == DLRM_OK) ix->singles_done = true;
    } else {
        rc = launch_interact_bwd_gather(ctx, tb->d_desc, tb->aligned16, tb->T, tb->dtype, indices, itype, table_stride,
                                        index_base, 1, d, batch, x, x_ld, dout, dout_ld, dx, dx_ld, dt, dt_ld, nullptr, tb->h_desc.data());
    }
    if (rc || (flags & DLRM_STEP_BWD_ONLY)) return rc;
    // once-hit rows: updated by the split backward, else by this apply (an unsplit indexer lists
    // them as chunks)
    const SinglesArgs sa{(ix->split && !split_bwd) ? ix->dev.single : nullptr, indices, itype, table_stride,
                         index_base, batch};
    return launch_sgd_apply(ctx, ix->dev, tb->d_desc, tb->aligned16, tb->T, tb->D, tb->dtype, 1, (int64_t)batch, dt,
                            DLRM_F32, dt_ld, d, lr, sa, prep);
}

int dlrm_step_bwd(dlrm_ctx* ctx, dlrm_tables* tb, dlrm_indexer* ix, const void* indices, int itype,
                  int64_t table_stride, int index_base, int batch, const void* x, int64_t x_ld, const void* dout,
                  int64_t dout_ld, int padding, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld, float lr,
                  unsigned flags) {
    return step_bwd_impl(ctx, tb, ix, indices, itype, table_stride, index_base, batch, x, x_ld, dout, dout_ld, padding,
                         dx, dx_ld, dt, dt_ld, lr, flags, nullptr);
}

int dlrm_step_bwd_prepare(dlrm_ctx* ctx, dlrm_tables* tb, dlrm_indexer* ix, const void* indices, int itype,
                          int64_t table_stride, int index_base, int batch, const void* x, int64_t x_ld,
                          const void* dout, int64_t dout_ld, int padding, float* dx, int64_t dx_ld, float* dt,
                          int64_t dt_ld, float lr, dlrm_indexer* next, const void* next_indices, unsigned flags) {
    CHECK_ARG(ctx && tb && ix && next && next != ix, "dlrm_step_bwd_prepare: null or shared indexer");
    CHECK_ARG(next->T == tb->T && batch <= next->dev.cap, "dlrm_step_bwd_prepare: next indexer too small");
    int rc = check_indices(ctx, tb, next_indices, itype, table_stride, batch, 1);
    if (rc) return rc;
    // the next batch's build runs as extra workgroups of this step's apply launch: the step
    // forward's split build (the same parts), so the next dlrm_step_fwd only gathers
    const int NB = (tb->T + 1 + 15) / 16;
    // (the split backward's shapes only: the apply launch that carries the build has no once-hit items)
    const bool inapply = batch > 0 && tb->T > 0 && batch <= kWaveApplyMaxN && NB <= 2 && tb->aligned16 &&
                         wave_fits(next, batch) &&
                         step_split_supported(tb->aligned16, tb->T, tb->dtype, tb->D, x, x_ld);
    if (!inapply)  // no pipelined form for this shape: the plain step (the next forward builds)
        return step_bwd_impl(ctx, tb, ix, indices, itype, table_stride, index_base, batch, x, x_ld, dout, dout_ld,
                             padding, dx, dx_ld, dt, dt_ld, lr, flags, nullptr);
    if (flags & DLRM_STEP_BWD_ONLY)  // (the next build rides on the apply launch)
        return step_bwd_impl(ctx, tb, ix, indices, itype, table_stride, index_base, batch, x, x_ld, dout, dout_ld,
                             padding, dx, dx_ld, dt, dt_ld, lr, flags, nullptr);
    next->built = false;
    next->prepared = false;
    // the wave build: 2^wave_parts_log2(batch) parts per table, one wave each (4 per workgroup)
    next->dev.vshift = wave_parts_log2(batch, next);
    if (next->dev.vshift < 2) next->dev.vshift = 2;
    const PrepArgs pa{next->dev, tb->d_desc, tb->T, next_indices, itype, table_stride, index_base, batch,
                      next->prep_err + 1};
    rc = step_bwd_impl(ctx, tb, ix, indices, itype, table_stride, index_base, batch, x, x_ld, dout, dout_ld, padding,
                       dx, dx_ld, dt, dt_ld, lr, flags, &pa);
    if (rc) return rc;
    record_build(next, true, next_indices, itype, table_stride, index_base, batch, 1);
    next->prepared = true;
    next->dev.has_map = 1;
    return DLRM_OK;
}

// ---- diagnostics: a native backtrace on a fatal signal (SIGSEGV / SIGBUS / SIGABRT), written to
// stderr before the previous handler runs (Python's faulthandler then prints the Python stack).
static struct sigaction g_prev[3];
static const int g_sigs[3] = {SIGSEGV, SIGBUS, SIGABRT};
static void fatal_trace(int sig, siginfo_t* si, void* uc) {
    static const char head[] = "\n[dlrm] fatal signal, native backtrace (innermost first):\n";
    (void)!write(2, head, sizeof head - 1);
    char line[96];
    const int n0 = snprintf(line, sizeof line, "[dlrm] signal %d, fault address %p\n", sig, si ? si->si_addr : nullptr);
    if (n0 > 0) (void)!write(2, line, (size_t)n0);
    void* fr[64];
    const int n = backtrace(fr, 64);
    backtrace_symbols_fd(fr, n, 2);
    for (int k = 0; k < 3; ++k)
        if (g_sigs[k] == sig) {
            sigaction(sig, &g_prev[k], nullptr);
            if (g_prev[k].sa_flags & SA_SIGINFO) {
                if (g_prev[k].sa_sigaction) {
                    g_prev[k].sa_sigaction(sig, si, uc);
                    return;
                }
            } else if (g_prev[k].sa_handler != SIG_DFL && g_prev[k].sa_handler != SIG_IGN) {
                g_prev[k].sa_handler(sig);
                return;
            }
        }
    signal(sig, SIG_DFL);
    raise(sig);
}

int dlrm_debug_fatal_trace(int on) {
    if (on == 2) {  // report who owns the handlers now (dladdr of the installed function), then arm
        for (int k = 0; k < 3; ++k) {
            struct sigaction cur;
            if (sigaction(g_sigs[k], nullptr, &cur) != 0) continue;
            void* fn = (cur.sa_flags & SA_SIGINFO) ? (void*)cur.sa_sigaction : (void*)cur.sa_handler;
            Dl_info di;
            memset(&di, 0, sizeof di);
            const bool named = fn && dladdr(fn, &di) != 0;
            fprintf(stderr, "[dlrm] signal %d handler %p (%s in %s)\n", g_sigs[k], fn,
                    named && di.dli_sname ? di.dli_sname : "?", named && di.dli_fname ? di.dli_fname : "?");
        }
        fflush(stderr);
    }
    if (on) {  // an alternate signal stack for this thread: a stack overflow is a SIGSEGV too
        static char* alt = nullptr;
        if (!alt) alt = (char*)malloc(1 << 20);
        if (alt) {
            stack_t ss;
            memset(&ss, 0, sizeof ss);
            ss.ss_sp = alt;
            ss.ss_size = 1 << 20;
            (void)sigaltstack(&ss, nullptr);
        }
    }
    for (int k = 0; k < 3; ++k) {
        if (on) {
            struct sigaction sa, old;
            memset(&sa, 0, sizeof sa);
            sa.sa_sigaction = fatal_trace;
            sa.sa_flags = SA_SIGINFO | SA_RESETHAND | SA_ONSTACK;
            sigemptyset(&sa.sa_mask);
            if (sigaction(g_sigs[k], &sa, &old) != 0) return DLRM_E_ARG;
            // (re-arming keeps the handler found the first time: chaining to ourselves would recurse)
            if (!((old.sa_flags & SA_SIGINFO) && old.sa_sigaction == fatal_trace)) g_prev[k] = old;
        } else {
            sigaction(g_sigs[k], &g_prev[k], nullptr);
        }
    }
    return DLRM_OK;
}

}  // extern "C"
