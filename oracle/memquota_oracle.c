/* ORACLE (test infrastructure only) -- C restatement of Mixer's memquota adapter, for the bench's
 * CPU baseline and as a second restatement the tests check against oracle/memquota.py.
 *
 *   rollingWindow  mixer/adapter/memquota/rollingWindow.go:21-113 (alloc :49-66, release :68-96,
 *                  roll :98-113)
 *   alloc / free   mixer/adapter/memquota/memquota.go:119-171 (alloc), :173-214 (free): cells for
 *                  ValidDuration 0, rolling windows of ceil(ValidDuration / 1s) * ticksPerSecond
 *                  ticks otherwise; best effort grabs what is left; a free of an absent cell or
 *                  window returns 0; a window whose slots are all free again is dropped
 *   HandleQuota    memquota.go:107-117 (amount > 0 alloc, < 0 free, 0 nothing)
 *   ticks          dedup.go:51-55 (ticksPerSecond 10, currentTick = UnixNano / nanosPerTick)
 *
 * Keys are independent and each key's requests are sequential (the reference serialises them on
 * its mutex in arrival order), so a batch is bucketed by key (stable) and the keys are handled in
 * parallel, one thread per key at a time (OpenMP).  int64 arithmetic wraps as Go's does.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MQ_TICKS_PER_SECOND 10
#define MQ_NANOS_PER_TICK (1000000000LL / MQ_TICKS_PER_SECOND)

static inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

typedef struct {
    int64_t max_amount, valid_ns;
    int64_t in_use;     /* cell (valid_ns == 0) */
    int live;           /* a cell in the map / a window in the map */
    int64_t avail;      /* window */
    int64_t *slots;
    int64_t nslots, cur, cur_tick;
} mq_key;

typedef struct {
    int64_t nkeys;
    mq_key *k;
} mq_state;

mq_state *mq_create(int64_t nkeys, const int64_t *max_amount, const int64_t *valid_ns) {
    mq_state *s = (mq_state *)calloc(1, sizeof(mq_state));
    if (!s) return NULL;
    s->nkeys = nkeys;
    s->k = (mq_key *)calloc((size_t)(nkeys > 0 ? nkeys : 1), sizeof(mq_key));
    if (!s->k) {
        free(s);
        return NULL;
    }
    for (int64_t i = 0; i < nkeys; i++) {
        s->k[i].max_amount = max_amount[i];
        s->k[i].valid_ns = valid_ns[i];
        if (valid_ns[i] != 0) {
            const int64_t seconds = (valid_ns[i] + 1000000000LL - 1) / 1000000000LL;
            s->k[i].nslots = seconds * MQ_TICKS_PER_SECOND;
            s->k[i].slots = (int64_t *)calloc((size_t)s->k[i].nslots, sizeof(int64_t));
        }
    }
    return s;
}

void mq_destroy(mq_state *s) {
    if (!s) return;
    for (int64_t i = 0; i < s->nkeys; i++) free(s->k[i].slots);
    free(s->k);
    free(s);
}

/* rollingWindow.go:98-113 */
static void w_roll(mq_key *w, int64_t tick) {
    int64_t behind = tick - w->cur_tick;
    if (behind > w->nslots) behind = w->nslots;
    for (int64_t i = 0; i < behind; i++) {
        const int64_t idx = (w->cur + 1 + i) % w->nslots;
        w->avail = wadd(w->avail, w->slots[idx]);
        w->slots[idx] = 0;
    }
    w->cur = (w->cur + behind) % w->nslots;  /* (Go's %: truncated, as C's) */
    w->cur_tick = tick;
}

/* rollingWindow.go:49-66 */
static int w_alloc(mq_key *w, int64_t amount, int64_t tick) {
    w_roll(w, tick);
    if (amount > w->avail) return 0;
    w->slots[w->cur] = wadd(w->slots[w->cur], amount);
    w->avail = wsub(w->avail, amount);
    return 1;
}

/* rollingWindow.go:68-96 */
static int64_t w_release(mq_key *w, int64_t amount, int64_t tick) {
    w_roll(w, tick);
    int64_t total = 0, idx = w->cur;
    for (int64_t i = 0; i < w->nslots; i++) {
        const int64_t av = w->slots[idx];
        if (av >= amount) {
            w->slots[idx] = wsub(w->slots[idx], amount);
            total = wadd(total, amount);
            break;
        }
        w->slots[idx] = 0;
        total = wadd(total, av);
        amount = wsub(amount, av);
        if (--idx < 0) idx = w->nslots - 1;
    }
    w->avail = wadd(w->avail, total);
    return total;
}

static void w_open(mq_key *w) {  /* newRollingWindow(limit, ticks) */
    w->live = 1;
    w->avail = w->max_amount;
    memset(w->slots, 0, (size_t)w->nslots * sizeof(int64_t));
    w->cur = 0;
    w->cur_tick = 0;
}

/* memquota.go:107-214 for one request of key k */
static int64_t mq_handle1(mq_key *k, int64_t amount, int best_effort, int64_t now_ns) {
    const int64_t tick = now_ns / MQ_NANOS_PER_TICK;
    if (amount > 0) {
        int64_t result = amount;
        if (k->valid_ns == 0) {
            const int64_t in_use = k->live ? k->in_use : 0;
            if (result > wsub(k->max_amount, in_use)) {
                if (!best_effort) return 0;
                result = wsub(k->max_amount, in_use);
            }
            k->in_use = wadd(in_use, result);
            k->live = 1;
            return result;
        }
        if (!k->live) w_open(k);
        if (!w_alloc(k, result, tick)) {
            if (!best_effort) return 0;
            result = k->avail;
            w_alloc(k, result, tick);
        }
        return result;
    }
    if (amount < 0) {
        const int64_t r = wsub(0, amount);
        if (k->valid_ns == 0) {
            const int64_t in_use = k->live ? k->in_use : 0;
            if (r >= in_use) {
                k->live = 0;
                k->in_use = 0;
                return in_use;
            }
            k->in_use = wsub(in_use, r);
            return r;
        }
        if (!k->live) return 0;
        const int64_t result = w_release(k, r, tick);
        if (k->avail == k->max_amount) k->live = 0;
        return result;
    }
    return 0;
}

/* One batch in arrival order: granted[i] for every request; keys outside [0, nkeys) are granted 0.
 * Returns 0, or -1 on allocation failure. */
int mq_handle_batch(mq_state *s, int64_t n, const int32_t *keys, const int64_t *amounts, const uint8_t *best_effort,
                    int64_t now_ns, int64_t *granted, int threads) {
    const int64_t K = s->nkeys;
    int64_t *start = (int64_t *)calloc((size_t)K + 2, sizeof(int64_t));
    int64_t *order = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    if (!start || !order) {
        free(start);
        free(order);
        return -1;
    }
    for (int64_t i = 0; i < n; i++) {  /* stable bucketing by key */
        const int32_t k = keys[i];
        if (k >= 0 && k < K) start[k + 2]++;
        else granted[i] = 0;
    }
    for (int64_t k = 0; k < K; k++) start[k + 2] += start[k + 1];
    for (int64_t i = 0; i < n; i++) {
        const int32_t k = keys[i];
        if (k >= 0 && k < K) order[start[k + 1]++] = i;
    }
    /* start[k] .. start[k + 1]: key k's requests in arrival order */
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads > 0 ? threads : 1)
    for (int64_t k = 0; k < K; k++)
        for (int64_t j = start[k]; j < start[k + 1]; j++) {
            const int64_t i = order[j];
            granted[i] = mq_handle1(&s->k[k], amounts[i], best_effort[i] != 0, now_ns);
        }
    free(start);
    free(order);
    return 0;
}
