// quota.cpp -- batched memquota host side (include/mxp.h; kernels in quota.hip).
//
// Reference: mixer/adapter/memquota/memquota.go (HandleQuota, alloc, free), rollingWindow.go,
// dedup.go (ticksPerSecond = 10, currentTick = now.UnixNano() / nanosPerTick).  The caller resolves
// each request's quota key (makeKey(instance.Name, instance.Dimensions)) to a dense key id and the
// key's limit (limit(): the first override whose dimensions match, else the default), and keeps
// DeduplicationID handling (handleDedup) -- the engine owns the per-key state and the arithmetic.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "engine_impl.h"
#include "quota_args.h"

extern "C" hipError_t mxp_quota_sort(void* tmp, size_t* tmp_bytes, const uint32_t* key, uint32_t n_keys,
                                     uint32_t* keys_in, uint32_t* keys_out, uint32_t* idx_in, uint32_t* idx_out,
                                     uint32_t n, int bits, hipStream_t s);
extern "C" uint32_t mxp_quota_piece_waves(uint32_t n);
extern "C" size_t mxp_quota_bucket_words(uint32_t n, uint32_t n_keys);
extern "C" hipError_t mxp_launch_quota(const mxp_quota_args* a, uint32_t* bucketed,
                                       hipStream_t s);

struct mxp_quota {
    uint32_t n_keys = 0;
    DevBuf max_amount, ticks, cells, avail, win_cur, win_tick, slot_off, slots;
    DevBuf keys_clamped, keys_sorted, idx_in, order, seg_start, tmp, samt, sbe, big, prec, done;
    size_t cap = 0, tmp_bytes = 0, radix_cap = 0, bucket_cap = 0;  // (tmp: the radix sort's or the bucketing's)
};

constexpr uint32_t kMaxBins = 4096;  // keys + the sentinel bucketed in LDS (quota.hip mxp_quota_hist)

extern "C" {

int mxp_quota_create(mxp_engine* eng, uint32_t n_keys, const int64_t* max_amount, const int64_t* valid_duration_ns,
                     mxp_quota** out) {
    if (!eng || !out || (n_keys && (!max_amount || !valid_duration_ns))) return MXP_ERR_ARG;
    if (eng->device < 0) return eng->fail(MXP_ERR_STATE, "host-only engine");
    hipError_t e;
    if ((e = hipSetDevice(eng->device)) != hipSuccess) return eng->hipfail(e, "hipSetDevice");
    std::unique_ptr<mxp_quota> Q(new mxp_quota());
    Q->n_keys = n_keys;
    std::vector<uint32_t> ticks(n_keys);
    std::vector<uint64_t> off(n_keys + 1, 0);
    for (uint32_t k = 0; k < n_keys; k++) {
        // newRollingWindow(limit, seconds * ticksPerSecond), seconds = ceil(ValidDuration / 1s)
        const int64_t vd = valid_duration_ns[k];
        ticks[k] = vd <= 0 ? 0u : (uint32_t)((vd + 999999999) / 1000000000) * 10u;
        off[k + 1] = off[k] + ticks[k];
    }
    std::vector<int64_t> zero64(n_keys, 0), avail(max_amount, max_amount + n_keys);
    std::vector<uint32_t> zero32(n_keys, 0);
    auto put = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.alloc(bytes ? bytes : 16)) != hipSuccess) return eng->hipfail(e, what);
        if (bytes && (e = hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice)) != hipSuccess) return eng->hipfail(e, what);
        return MXP_OK;
    };
    int rc;
    if ((rc = put(Q->max_amount, max_amount, n_keys * 8, "quota max"))) return rc;
    if ((rc = put(Q->ticks, ticks.data(), n_keys * 4, "quota ticks"))) return rc;
    if ((rc = put(Q->cells, zero64.data(), n_keys * 8, "quota cells"))) return rc;
    if ((rc = put(Q->avail, avail.data(), n_keys * 8, "quota avail"))) return rc;
    if ((rc = put(Q->win_cur, zero32.data(), n_keys * 4, "quota cur"))) return rc;
    if ((rc = put(Q->win_tick, zero64.data(), n_keys * 8, "quota tick"))) return rc;
    if ((rc = put(Q->slot_off, off.data(), off.size() * 8, "quota slot_off"))) return rc;
    if ((e = Q->slots.alloc(off[n_keys] * 8 + 16)) != hipSuccess) return eng->hipfail(e, "quota slots");
    if ((e = hipMemset(Q->slots.p, 0, off[n_keys] * 8 + 16)) != hipSuccess) return eng->hipfail(e, "quota slots");
    // segments of keys 0 .. n_keys (the last: out-of-range key ids, mxp_quota_clamp), plus the end
    if ((e = Q->seg_start.alloc(((size_t)n_keys + 2) * 4)) != hipSuccess) return eng->hipfail(e, "quota seg");
    // long keys' pieces: per-key flags and finished counters (the kernel leaves the counters at 0)
    if ((e = Q->big.alloc(((size_t)n_keys + 1) * 4)) != hipSuccess) return eng->hipfail(e, "quota flags");
    if ((e = Q->done.alloc(((size_t)n_keys + 1) * 4)) != hipSuccess) return eng->hipfail(e, "quota counters");
    if ((e = hipMemset(Q->done.p, 0, ((size_t)n_keys + 1) * 4)) != hipSuccess) return eng->hipfail(e, "quota counters");
    *out = Q.release();
    return MXP_OK;
}

void mxp_quota_destroy(mxp_engine* eng, mxp_quota* q) {
    if (eng && eng->device >= 0) (void)hipSetDevice(eng->device);
    delete q;
}

int mxp_quota_alloc_device(mxp_engine* eng, mxp_quota* Q, uint32_t n, const uint32_t* d_key, const int64_t* d_amount,
                           const uint8_t* d_best_effort, int64_t now_ns, void* stream, int64_t* d_granted,
                           int64_t* d_delta) {
    if (!eng || !Q || (n && (!d_key || !d_amount || !d_best_effort || !d_granted))) return MXP_ERR_ARG;
    if (!n || !Q->n_keys) return MXP_OK;
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    hipError_t e;
    // up to kMaxBins - 1 keys: bucketed by a counting sort in the launch (MXP_QUOTA_RADIX=1 forces the
    // radix sort path, for tests); else a radix sort of (key, arrival index) pairs first
    const char* force_radix = getenv("MXP_QUOTA_RADIX");
    const bool bucketed = Q->n_keys + 1 <= kMaxBins && !(force_radix && *force_radix == '1');
    if (n > Q->cap) {
        if ((e = Q->keys_sorted.alloc((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "quota keys");
        if ((e = Q->order.alloc((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "quota order");
        if ((e = Q->samt.alloc((size_t)n * 8)) != hipSuccess) return eng->hipfail(e, "quota sorted amounts");
        if ((e = Q->sbe.alloc((size_t)n)) != hipSuccess) return eng->hipfail(e, "quota sorted flags");
        if ((e = Q->prec.alloc(((size_t)Q->n_keys + 1 + mxp_quota_piece_waves(n)) * 48)) != hipSuccess)
            return eng->hipfail(e, "quota piece records");
        Q->cap = n;
        Q->radix_cap = 0;
        Q->bucket_cap = 0;
    }
    if (bucketed && Q->bucket_cap < n) {
        if ((e = Q->tmp.alloc(mxp_quota_bucket_words(n, Q->n_keys) * 4)) != hipSuccess)
            return eng->hipfail(e, "quota bucket scratch");
        Q->bucket_cap = n;
        Q->radix_cap = 0;
    }
    if (!bucketed) {
        if (Q->radix_cap < n) {
            if ((e = Q->keys_clamped.alloc((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "quota keys");
            if ((e = Q->idx_in.alloc((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "quota idx");
            size_t need = 0;
            if ((e = mxp_quota_sort(nullptr, &need, nullptr, 0, nullptr, nullptr, nullptr, nullptr, n, 32, s)) != hipSuccess)
                return eng->hipfail(e, "quota sort size");
            if ((e = Q->tmp.alloc(need)) != hipSuccess) return eng->hipfail(e, "quota sort tmp");
            Q->tmp_bytes = need;
            Q->radix_cap = n;
            Q->bucket_cap = 0;
        }
        // sort keys 0 .. n_keys (n_keys = the sentinel of out-of-range ids): enough bits for n_keys itself
        int bits = 1;
        while (bits < 32 && (1ull << bits) <= Q->n_keys) bits++;
        size_t tb = Q->tmp_bytes;
        if ((e = mxp_quota_sort(Q->tmp.p, &tb, d_key, Q->n_keys, Q->keys_clamped.as<uint32_t>(),
                                Q->keys_sorted.as<uint32_t>(), Q->idx_in.as<uint32_t>(), Q->order.as<uint32_t>(), n,
                                bits, s)) != hipSuccess)
            return eng->hipfail(e, "quota sort");
    }
    mxp_quota_args A;
    memset(&A, 0, sizeof A);
    A.n = n;
    A.n_keys = Q->n_keys;
    A.tick = now_ns / 100000000;  // nanosPerTick = 1e9 / ticksPerSecond
    A.key = d_key;
    A.amount = d_amount;
    A.best_effort = d_best_effort;
    A.order = Q->order.as<uint32_t>();
    A.samt = Q->samt.as<int64_t>();
    A.sbe = Q->sbe.as<uint8_t>();
    A.seg_start = Q->seg_start.as<uint32_t>();
    A.skeys = Q->keys_sorted.as<uint32_t>();
    A.big = Q->big.as<uint32_t>();
    A.prec = Q->prec.as<int64_t>();
    A.done = Q->done.as<uint32_t>();
    A.granted = d_granted;
    A.delta = d_delta;
    A.max_amount = Q->max_amount.as<int64_t>();
    A.ticks = Q->ticks.as<uint32_t>();
    A.cells = Q->cells.as<int64_t>();
    A.avail = Q->avail.as<int64_t>();
    A.win_cur = Q->win_cur.as<uint32_t>();
    A.win_tick = Q->win_tick.as<int64_t>();
    A.slot_off = Q->slot_off.as<uint64_t>();
    A.slots = Q->slots.as<int64_t>();
    // debug: MXP_QUOTA_PROF=<file> appends each wave's time (100 MHz ticks), run steps, shader
    // clocks in all and in the 32-bit replays (waves 0 .. n_keys: the keys' first pieces)
    const char* prof_path = getenv("MXP_QUOTA_PROF");
    DevBuf prof;
    if (prof_path && *prof_path) {
        if ((e = prof.alloc(((size_t)Q->n_keys + 1 + mxp_quota_piece_waves(n)) * 32)) != hipSuccess ||
            (e = hipMemsetAsync(prof.p, 0, ((size_t)Q->n_keys + 1 + mxp_quota_piece_waves(n)) * 32, s)) != hipSuccess)
            return eng->hipfail(e, "quota prof");
        A.prof = prof.as<int64_t>();
    }
    if ((e = mxp_launch_quota(&A, bucketed ? Q->tmp.as<uint32_t>() : nullptr, s)) != hipSuccess)
        return eng->hipfail(e, "launch quota");
    if (A.prof) {
        const uint32_t waves = Q->n_keys + 1 + mxp_quota_piece_waves(n);
        std::vector<int64_t> h((size_t)waves * 4);
        if ((e = hipMemcpyAsync(h.data(), A.prof, h.size() * 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return eng->hipfail(e, "quota prof");
        if (FILE* f = fopen(prof_path, "a")) {
            for (uint32_t k = 0; k < waves; k++) fprintf(f, "%u %lld %lld %lld %lld\n", k, (long long)h[4 * k], (long long)h[4 * k + 1],
                                                          (long long)h[4 * k + 2], (long long)h[4 * k + 3]);
            fclose(f);
        }
    }
    return MXP_OK;
}

int mxp_quota_alloc(mxp_engine* eng, mxp_quota* Q, uint32_t n, const uint32_t* key, const int64_t* amount,
                    const uint8_t* best_effort, int64_t now_ns, int64_t* granted) {
    if (!eng || !Q || (n && (!key || !amount || !best_effort || !granted))) return MXP_ERR_ARG;
    if (!n) return MXP_OK;
    for (uint32_t i = 0; i < n; i++)
        if (key[i] >= Q->n_keys) return eng->fail(MXP_ERR_ARG, "quota key id out of range");
    hipError_t e;
    if ((e = hipSetDevice(eng->device)) != hipSuccess) return eng->hipfail(e, "hipSetDevice");
    DevBuf dk, da, db, dg;
    if ((e = dk.alloc((size_t)n * 4)) != hipSuccess || (e = da.alloc((size_t)n * 8)) != hipSuccess ||
        (e = db.alloc(n)) != hipSuccess || (e = dg.alloc((size_t)n * 8)) != hipSuccess)
        return eng->hipfail(e, "quota buffers");
    if ((e = hipMemcpyAsync(dk.p, key, (size_t)n * 4, hipMemcpyHostToDevice, eng->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(da.p, amount, (size_t)n * 8, hipMemcpyHostToDevice, eng->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(db.p, best_effort, n, hipMemcpyHostToDevice, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "quota upload");
    int rc = mxp_quota_alloc_device(eng, Q, n, dk.as<uint32_t>(), da.as<int64_t>(), db.as<uint8_t>(), now_ns,
                                    eng->stream, dg.as<int64_t>(), nullptr);
    if (rc) return rc;
    return eng->download(granted, dg.p, (size_t)n * 8, "quota download");  // (synchronises)
}

}  // extern "C"
