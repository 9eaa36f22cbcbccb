// dac.hip — the Criteo DAC data path (SURVEY §8 rows f2 + f4), native:
//   host:   parseline / binarize (criteo.jl:137-176): TSV -> 160-B DACRecords
//           categorical_values + reindex / reindex! (criteo.jl:182-262): per-feature value -> id
//           maps in first-appearance order, shard after shard
//   device: load! (criteo.jl:284-307) as a decode kernel: a batch of raw records uploaded as one
//           contiguous block is split into labels [B] f32, dense [B][13] f32 and the sparse
//           indices [26][B] (the hot path's table-major index layout, criteo.jl:324) in HBM.
#include <math.h>
#include <string.h>

#include <new>
#include <unordered_map>
#include <vector>

#include "common.hpp"

static_assert(sizeof(dlrm_dac_record) == 160, "DACRecord is 160 bytes (criteo.jl:91-95)");

namespace dlrm {

// ---------------------------------------------------------------------- decode (load!)
// One thread per (record, 4-byte word): the 40 words of a record are read coalesced, then each
// word goes to its destination (label -> f32, continuous -> dense row, categorical -> [t][b]).
__global__ void dac_decode_kernel(const uint32_t* __restrict__ rec, int B, float* __restrict__ labels,
                                  float* __restrict__ dense, int64_t dense_ld, void* __restrict__ sparse, int itype,
                                  int64_t tstride) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)B * 40) return;
    const int b = (int)(i / 40), w = (int)(i % 40);
    const uint32_t v = rec[i];
    if (w == 0) {
        labels[b] = (float)(int32_t)v;  // labels[i] = record.label (Int32 -> Float32)
    } else if (w <= 13) {
        dense[(int64_t)b * dense_ld + (w - 1)] = __uint_as_float(v);
    } else {
        const int t = w - 14;
        if (itype == DLRM_I64)
            ((int64_t*)sparse)[t * tstride + b] = (int64_t)v;
        else
            ((uint32_t*)sparse)[t * tstride + b] = v;
    }
}

int launch_dac_decode(dlrm_ctx* ctx, const void* rec, int B, float* labels, float* dense, int64_t dense_ld,
                      void* sparse, int itype, int64_t tstride) {
    if (B == 0) return DLRM_OK;
    const int64_t n = (int64_t)B * 40;
    hipLaunchKernelGGL(dac_decode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx_stream(ctx),
                       (const uint32_t*)rec, B, labels, dense, dense_ld, sparse, itype, tstride);
    return ctx_hip(ctx, hipGetLastError(), "dac_decode launch");
}

}  // namespace dlrm

// ---------------------------------------------------------------------- host: parseline
namespace {

// emptyparse(T, str; base) (criteo.jl:41-47): empty field -> 0, else parse; false on a bad field
bool parse_int(const char* s, const char* e, int base, bool is_signed, int64_t* out) {
    if (s == e) {
        *out = 0;
        return true;
    }
    bool neg = false;
    if (*s == '+' || *s == '-') {
        if (!is_signed && *s == '-') return false;
        neg = *s == '-';
        ++s;
        if (s == e) return false;
    }
    int64_t v = 0;
    for (; s < e; ++s) {
        int d;
        const char c = *s;
        if (c >= '0' && c <= '9') d = c - '0';
        else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
        else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
        else return false;
        if (d >= base) return false;
        v = v * base + d;
        if (v > 0xffffffffll) return false;
    }
    *out = neg ? -v : v;
    return true;
}

}  // namespace

extern "C" int dlrm_dac_parse_tsv(const char* text, int64_t len, dlrm_dac_record* out, int64_t cap, int64_t* count) {
    if (!count || (len > 0 && !text) || cap < 0 || (cap > 0 && !out)) return DLRM_E_ARG;
    int64_t n = 0;
    const char* p = text;
    const char* end = text + len;
    while (p < end) {
        const char* eol = (const char*)memchr(p, '\n', (size_t)(end - p));
        if (!eol) eol = end;
        if (eol == p) {  // blank line (e.g. a trailing newline): no record
            p = eol + 1;
            continue;
        }
        if (n >= cap) return DLRM_E_NOMEM;
        dlrm_dac_record& r = out[n];
        const char* f = p;
        for (int k = 0; k < 40; ++k) {
            const char* fe = (const char*)memchr(f, '\t', (size_t)(eol - f));
            if (k == 39) {
                if (fe) return DLRM_E_ARG;  // more than 40 fields
                fe = eol;
            } else if (!fe) {
                return DLRM_E_ARG;  // fewer than 40 fields
            }
            const char* fe_trim = fe;
            if (k == 39 && fe_trim > f && fe_trim[-1] == '\r') --fe_trim;
            int64_t v;
            if (k == 0) {  // label: parse(Int32, ...; base = 10), never empty
                if (f == fe_trim || !parse_int(f, fe_trim, 10, true, &v)) return DLRM_E_ARG;
                if (v < INT32_MIN || v > INT32_MAX) return DLRM_E_ARG;  // parse(Int32, ...) throws OverflowError
                r.label = (int32_t)v;
            } else if (k <= 13) {  // logtransform(emptyparse(Int32, ...; base = 10))
                if (!parse_int(f, fe_trim, 10, true, &v) || v < INT32_MIN || v > INT32_MAX) return DLRM_E_ARG;
                const float x = (float)(int32_t)v;
                r.continuous[k - 1] = logf(fmaxf(x, 0.0f) + 1.0f);  // criteo.jl:55, Float32
            } else {  // emptyparse(UInt32, ...; base = 16)
                if (!parse_int(f, fe_trim, 16, false, &v)) return DLRM_E_ARG;
                r.categorical[k - 14] = (uint32_t)v;
            }
            f = fe + 1;
        }
        ++n;
        p = eol + 1;
    }
    *count = n;
    return DLRM_OK;
}

// ---------------------------------------------------------------------- host: reindex maps
struct dlrm_dac_maps {
    std::unordered_map<uint32_t, uint32_t> map[26];
};

extern "C" int dlrm_dac_maps_create(dlrm_dac_maps** out) {
    if (!out) return DLRM_E_ARG;
    *out = new (std::nothrow) dlrm_dac_maps();
    return *out ? DLRM_OK : DLRM_E_NOMEM;
}

extern "C" int dlrm_dac_maps_destroy(dlrm_dac_maps* m) {
    delete m;
    return DLRM_OK;
}

// categorical_values (OrderedSet per feature, in record order) followed by reindex! (get!(dict,
// v, length(dict) + 1)): a value seen for the first time gets the next id, 1-based.  Feeding
// shards in order gives the monolithic maps (the reference's test/data/criteo.jl property).
extern "C" int dlrm_dac_maps_add(dlrm_dac_maps* m, const dlrm_dac_record* recs, int64_t n) {
    if (!m || n < 0 || (n > 0 && !recs)) return DLRM_E_ARG;
    for (int j = 0; j < 26; ++j) {
        auto& d = m->map[j];
        for (int64_t i = 0; i < n; ++i) {
            const uint32_t v = recs[i].categorical[j];
            d.emplace(v, (uint32_t)(d.size() + 1));
        }
    }
    return DLRM_OK;
}

extern "C" int dlrm_dac_maps_sizes(const dlrm_dac_maps* m, int64_t* sizes) {
    if (!m || !sizes) return DLRM_E_ARG;
    for (int j = 0; j < 26; ++j) sizes[j] = (int64_t)m->map[j].size();
    return DLRM_OK;
}

extern "C" int dlrm_dac_maps_lookup(const dlrm_dac_maps* m, int feature, uint32_t value, uint32_t* id) {
    if (!m || !id || feature < 0 || feature >= 26) return DLRM_E_ARG;
    const auto it = m->map[feature].find(value);
    if (it == m->map[feature].end()) return DLRM_E_INDEX;
    *id = it->second;
    return DLRM_OK;
}

// reindex!(data, maps) (criteo.jl:251-259): categorical[j] <- maps[j][categorical[j]] in place.
// A value missing from a map is a KeyError in the reference: DLRM_E_INDEX, records untouched
// from the failing one on.
extern "C" int dlrm_dac_reindex(const dlrm_dac_maps* m, dlrm_dac_record* recs, int64_t n) {
    if (!m || n < 0 || (n > 0 && !recs)) return DLRM_E_ARG;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t ids[26];
        for (int j = 0; j < 26; ++j) {
            const auto it = m->map[j].find(recs[i].categorical[j]);
            if (it == m->map[j].end()) return DLRM_E_INDEX;
            ids[j] = it->second;
        }
        memcpy(recs[i].categorical, ids, sizeof(ids));
    }
    return DLRM_OK;
}

// ---------------------------------------------------------------------- native prefetching loader
// DACLoader's iteration with a native prefetch thread: the worker copies batch i's records into
// one of two pinned (hipHostMalloc) buffers, uploads them on the loader's own stream and decodes
// them into the caller's slot-i&1 outputs, while the caller computes on the other slot.  The
// caller's stream waits for a slot's `ready` event (dlrm_dac_loader_next); releasing a slot
// records `consumed` on the caller's stream, which the worker's stream waits for before it
// overwrites that slot.  The worker has its own dlrm_ctx (a ctx is not re-entrant).
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

struct dlrm_dac_loader {
    int device = 0;
    dlrm_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    const char* data = nullptr;
    int64_t count = 0;
    int B = 0, itype = 0;
    void* pinned[2] = {nullptr, nullptr};
    void* raw[2] = {nullptr, nullptr};
    float* labels[2] = {nullptr, nullptr};
    float* dense[2] = {nullptr, nullptr};
    void* sparse[2] = {nullptr, nullptr};
    hipEvent_t ready[2] = {}, consumed[2] = {}, h2d[2] = {};
    bool consumed_valid[2] = {false, false}, h2d_valid[2] = {false, false};
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool slot_free[2] = {true, true};
    bool held[2] = {false, false};  // handed to the caller by next, not yet released
    std::deque<int> ready_q;
    int64_t produced = 0, nbatches = 0;
    bool stop = false, running = false;
    int error = 0;
};

namespace {

void dac_worker(dlrm_dac_loader* L) {
    if (hipSetDevice(L->device) != hipSuccess) {
        std::lock_guard<std::mutex> g(L->mu);
        L->error = DLRM_E_HIP;
        L->cv.notify_all();
        return;
    }
    const size_t bytes = (size_t)L->B * sizeof(dlrm_dac_record);
    for (int64_t i = 0; i < L->nbatches; ++i) {
        const int slot = (int)(i & 1);
        {
            std::unique_lock<std::mutex> lk(L->mu);
            L->cv.wait(lk, [&] { return L->stop || L->slot_free[slot]; });
            if (L->stop) return;
            L->slot_free[slot] = false;
        }
        int rc = DLRM_OK;
        if (L->h2d_valid[slot] && hipEventSynchronize(L->h2d[slot]) != hipSuccess) rc = DLRM_E_HIP;
        if (rc == DLRM_OK) {
            memcpy(L->pinned[slot], L->data + (size_t)i * bytes, bytes);
            if (L->consumed_valid[slot] && hipStreamWaitEvent(L->stream, L->consumed[slot], 0) != hipSuccess)
                rc = DLRM_E_HIP;
        }
        if (rc == DLRM_OK && hipMemcpyAsync(L->raw[slot], L->pinned[slot], bytes, hipMemcpyHostToDevice, L->stream) !=
                                 hipSuccess)
            rc = DLRM_E_HIP;
        if (rc == DLRM_OK && hipEventRecord(L->h2d[slot], L->stream) != hipSuccess) rc = DLRM_E_HIP;
        L->h2d_valid[slot] = rc == DLRM_OK;
        if (rc == DLRM_OK)
            rc = dlrm::launch_dac_decode(L->ctx, L->raw[slot], L->B, L->labels[slot], L->dense[slot], 13,
                                         L->sparse[slot], L->itype, L->B);
        if (rc == DLRM_OK && hipEventRecord(L->ready[slot], L->stream) != hipSuccess) rc = DLRM_E_HIP;
        std::lock_guard<std::mutex> g(L->mu);
        if (rc != DLRM_OK) {
            L->error = rc;
            L->cv.notify_all();
            return;
        }
        L->ready_q.push_back(slot);
        ++L->produced;
        L->cv.notify_all();
    }
}

void dac_loader_join(dlrm_dac_loader* L) {
    {
        std::lock_guard<std::mutex> g(L->mu);
        L->stop = true;
        L->cv.notify_all();
    }
    if (L->th.joinable()) L->th.join();
    L->running = false;
}

}  // namespace

extern "C" int dlrm_dac_loader_create(int device, const dlrm_dac_record* records, int64_t count, int batch,
                                      int itype, float* const* labels, float* const* dense, void* const* sparse,
                                      dlrm_dac_loader** out) {
    if (!out || batch <= 0 || count < 0 || (count > 0 && !records) || !labels || !dense || !sparse) return DLRM_E_ARG;
    if (itype != DLRM_I32 && itype != DLRM_I64) return DLRM_E_ARG;
    for (int k = 0; k < 2; ++k)
        if (!labels[k] || !dense[k] || !sparse[k]) return DLRM_E_ARG;
    dlrm_dac_loader* L = new (std::nothrow) dlrm_dac_loader();
    if (!L) return DLRM_E_NOMEM;
    L->device = device;
    L->data = (const char*)records;
    L->count = count;
    L->B = batch;
    L->itype = itype;
    const size_t bytes = (size_t)batch * sizeof(dlrm_dac_record);
    bool ok = hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) == hipSuccess;
    for (int k = 0; ok && k < 2; ++k) {
        L->labels[k] = labels[k];
        L->dense[k] = dense[k];
        L->sparse[k] = sparse[k];
        ok = hipHostMalloc(&L->pinned[k], bytes, hipHostMallocDefault) == hipSuccess &&
             hipMalloc(&L->raw[k], bytes) == hipSuccess &&
             hipEventCreateWithFlags(&L->ready[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&L->consumed[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&L->h2d[k], hipEventDisableTiming) == hipSuccess;
    }
    if (ok) ok = dlrm_ctx_create(device, L->stream, &L->ctx) == DLRM_OK;
    if (!ok) {
        dlrm_dac_loader_destroy(L);
        return DLRM_E_HIP;
    }
    *out = L;
    return DLRM_OK;
}

extern "C" int dlrm_dac_loader_start(dlrm_dac_loader* L, int64_t* nbatches) {
    if (!L) return DLRM_E_ARG;
    {
        // a slot the caller still holds may still be read on its stream: refilling it for a new
        // epoch would overwrite a live batch (and a second live iterator would share ready_q)
        std::lock_guard<std::mutex> g(L->mu);
        if (L->held[0] || L->held[1]) return DLRM_E_STATE;
    }
    dac_loader_join(L);  // a previous epoch's worker, if any
    // the previous epoch's uploads must have left the pinned buffers / raw slots
    if (L->stream && hipStreamSynchronize(L->stream) != hipSuccess) return DLRM_E_HIP;
    L->stop = false;
    L->error = 0;
    L->ready_q.clear();
    L->produced = 0;
    L->slot_free[0] = L->slot_free[1] = true;
    L->nbatches = L->count / L->B;  // whole batches only (criteo.jl:326-329)
    if (nbatches) *nbatches = L->nbatches;
    L->running = true;
    L->th = std::thread(dac_worker, L);
    return DLRM_OK;
}

extern "C" int dlrm_dac_loader_next(dlrm_dac_loader* L, void* consumer_stream, int* slot) {
    if (!L || !slot) return DLRM_E_ARG;
    int s;
    {
        std::unique_lock<std::mutex> lk(L->mu);
        L->cv.wait(lk, [&] { return !L->ready_q.empty() || L->error || !L->running || L->produced >= L->nbatches; });
        if (L->ready_q.empty()) {
            if (L->error) return L->error;
            *slot = -1;  // the epoch is over
            return DLRM_OK;
        }
        s = L->ready_q.front();
        L->ready_q.pop_front();
        L->held[s] = true;
    }
    if (hipStreamWaitEvent((hipStream_t)consumer_stream, L->ready[s], 0) != hipSuccess) return DLRM_E_HIP;
    *slot = s;
    return DLRM_OK;
}

extern "C" int dlrm_dac_loader_release(dlrm_dac_loader* L, int slot, void* consumer_stream) {
    if (!L || slot < 0 || slot > 1) return DLRM_E_ARG;
    if (hipEventRecord(L->consumed[slot], (hipStream_t)consumer_stream) != hipSuccess) return DLRM_E_HIP;
    std::lock_guard<std::mutex> g(L->mu);
    L->consumed_valid[slot] = true;
    L->held[slot] = false;
    L->slot_free[slot] = true;
    L->cv.notify_all();
    return DLRM_OK;
}

extern "C" int dlrm_dac_loader_stop(dlrm_dac_loader* L) {
    if (!L) return DLRM_E_ARG;
    dac_loader_join(L);
    return DLRM_OK;
}

extern "C" int dlrm_dac_loader_destroy(dlrm_dac_loader* L) {
    if (!L) return DLRM_OK;
    dac_loader_join(L);
    if (L->stream) (void)hipStreamSynchronize(L->stream);
    if (L->ctx) dlrm_ctx_destroy(L->ctx);
    for (int k = 0; k < 2; ++k) {
        if (L->pinned[k]) (void)hipHostFree(L->pinned[k]);
        if (L->raw[k]) (void)hipFree(L->raw[k]);
        if (L->ready[k]) (void)hipEventDestroy(L->ready[k]);
        if (L->consumed[k]) (void)hipEventDestroy(L->consumed[k]);
        if (L->h2d[k]) (void)hipEventDestroy(L->h2d[k]);
    }
    if (L->stream) (void)hipStreamDestroy(L->stream);
    delete L;
    return DLRM_OK;
}
