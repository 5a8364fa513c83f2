// group.cpp -- device groups (include/mxp_group.h): one engine per GPU behind one handle, request
// shards evaluated by every member at once, and the step's one all-reduce of hits[R] ++
// quota_delta[K] over RCCL.
//
// Reference: the cross-request state a sharded Check path has to sum is the per-Resolve metrics
// (mixer/pkg/runtime/resolver.go:123-138; the engine's per-rule hit counters stand for resolve_rules)
// and memquota's per-key state (mixer/adapter/memquota/memquota.go:43-52,107-118); everything else a
// request reads is its own bag and the immutable rule set (resolver.go:202-238).
//
// Threads: member 0's work runs on the calling thread, member k's on a crew thread of its own, each
// with its device current; a group call returns once every member has enqueued (or, for the host
// calls, finished) its part.  The calling thread's current device is restored on return.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <thread>

#include "../../include/mxp_group.h"
#include "engine_impl.h"

extern "C" hipError_t mxp_launch_group_fold(long long* total, long long* step, uint32_t n, hipStream_t s);

namespace {

// librccl, loaded on first use: libmxp itself does not depend on it (a host-only or one-GPU user
// never loads it).  When PyTorch already mapped its own librccl.so.1 the loader hands that one back
// (same soname): one RCCL per process.
struct Rccl {
    void* h = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    bool tried = false;
    std::string err;
    bool load() {
        if (tried) return h != nullptr;
        tried = true;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) {
            const char* e = dlerror();
            err = std::string("dlopen librccl: ") + (e ? e : "?");
            return false;
        }
        auto sym = [&](const char* s) {
            void* p = dlsym(h, s);
            if (!p) err = std::string("librccl lacks ") + s;
            return p;
        };
        CommInitAll = (decltype(CommInitAll))sym("ncclCommInitAll");
        CommDestroy = (decltype(CommDestroy))sym("ncclCommDestroy");
        AllReduce = (decltype(AllReduce))sym("ncclAllReduce");
        GroupStart = (decltype(GroupStart))sym("ncclGroupStart");
        GroupEnd = (decltype(GroupEnd))sym("ncclGroupEnd");
        GetErrorString = (decltype(GetErrorString))sym("ncclGetErrorString");
        if (!CommInitAll || !CommDestroy || !AllReduce || !GroupStart || !GroupEnd || !GetErrorString) {
            h = nullptr;
            return false;
        }
        return true;
    }
    std::string text(ncclResult_t r) const { return GetErrorString ? GetErrorString(r) : std::to_string((int)r); }
};
Rccl& rccl() {
    static Rccl* r = new Rccl();  // (never unloaded: communicators may outlive static destructors)
    return *r;
}
std::mutex g_rccl_mu;

// Persistent threads for members 1 .. n-1 (member 0 runs on the caller): one job at a time.
class Crew {
  public:
    explicit Crew(uint32_t n) : n_(n) {
        for (uint32_t k = 1; k < n; k++) th_.emplace_back([this, k] { loop(k); });
    }
    ~Crew() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(const std::function<void(uint32_t)>& f) {
        if (n_ <= 1) {
            f(0);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &f;
            left_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [&] { return left_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(uint32_t k) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(uint32_t)>* job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                job = job_;
            }
            (*job)(k);
            std::lock_guard<std::mutex> g(mu_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    uint32_t n_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t)>* job_ = nullptr;
    uint64_t gen_ = 0;
    uint32_t left_ = 0;
    bool stop_ = false;
};

// the calling thread's current device, restored when a group call returns
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) {
            (void)hipGetLastError();
            dev = -1;
        }
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

template <class T>
using PinnedVec = std::vector<T, PinnedAlloc<T>>;

// a fixed array of non-movable elements (DevBuf members), sized once
template <class T>
struct Fixed {
    std::unique_ptr<T[]> p;
    size_t n = 0;
    void resize(size_t k) {
        p.reset(new T[k]);
        n = k;
    }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    T* begin() { return p.get(); }
    T* end() { return p.get() + n; }
    size_t size() const { return n; }
};

}  // namespace

struct mxp_group {
    struct Member {
        mxp_engine* eng = nullptr;
        int device = 0;
        ncclComm_t comm = nullptr;
        DevBuf step, total;            // counters (total aliases step when nothing is reduced)
        DevBuf match, err, req_err;    // results of the last mxp_group_eval
        uint32_t eval_n = 0;
        bool eval_bitmap = false, evaluated = false;
        hipStream_t qs = nullptr;      // memquota stream (beside the evaluation)
        // the member's evaluation stream: non-blocking, so the engine's synchronous copies on the
        // legacy stream (a batch upload's, a pack's) never wait for a queued evaluation
        hipStream_t es = nullptr;
        hipEvent_t fork = nullptr, join = nullptr;
        bool q_pending = false;        // a quota replay on qs the main stream has not joined yet
        PinnedVec<int64_t> host_ctr;   // host reduction
        int rc = 0;
        std::string err_text;
        hipStream_t stream() const { return es ? es : eng->stream; }
    };
    Fixed<Member> m;
    std::unique_ptr<Crew> crew;
    int reduce = MXP_REDUCE_NONE;
    std::string last_error;
    uint32_t R = 0, K = 0;
    PinnedVec<int64_t> host_sum;
    std::vector<uint64_t> lo;          // member k's first global request of the last batch call; lo[n] = total
    // finder mode: member 0 asks the caller's finder, the others take the vocabulary it found
    bool finder = false;

    uint32_t size() const { return (uint32_t)m.size(); }
    int fail(int code, const std::string& msg) {
        last_error = msg;
        return code;
    }
    int hipfail(hipError_t e, const std::string& what) { return fail(MXP_ERR_DEVICE, what + ": " + hipGetErrorString(e)); }
    // f(k) on every member (device current, errors recorded per member); the first failure wins
    int each(const std::function<int(uint32_t)>& f) {
        for (auto& x : m) {
            x.rc = 0;
            x.err_text.clear();
        }
        crew->run([&](uint32_t k) {
            Member& x = m[k];
            hipError_t e = hipSetDevice(x.device);
            if (e != hipSuccess) {
                x.rc = MXP_ERR_DEVICE;
                x.err_text = std::string("hipSetDevice: ") + hipGetErrorString(e);
                return;
            }
            x.rc = f(k);
            if (x.rc && x.err_text.empty()) x.err_text = x.eng->last_error;
        });
        for (uint32_t k = 0; k < size(); k++)
            if (m[k].rc) return fail(m[k].rc, "member " + std::to_string(k) + ": " + m[k].err_text);
        return MXP_OK;
    }
    // allocate and zero the counters for the current (R, K)
    int reset_counters() {
        const size_t bytes = (size_t)std::max<uint32_t>(1, R + K) * 8;
        return each([&](uint32_t k) -> int {
            Member& x = m[k];
            hipError_t e;
            if (x.q_pending) {
                (void)hipEventSynchronize(x.join);
                x.q_pending = false;
            }
            if ((e = hipStreamSynchronize(x.stream())) != hipSuccess) return x.eng->hipfail(e, "sync");
            if ((e = x.step.reserve(bytes)) != hipSuccess) return x.eng->hipfail(e, "alloc step counters");
            if ((e = hipMemsetAsync(x.step.p, 0, bytes, x.stream())) != hipSuccess) return x.eng->hipfail(e, "zero counters");
            if (reduce != MXP_REDUCE_NONE) {
                if ((e = x.total.reserve(bytes)) != hipSuccess) return x.eng->hipfail(e, "alloc total counters");
                if ((e = hipMemsetAsync(x.total.p, 0, bytes, x.stream())) != hipSuccess) return x.eng->hipfail(e, "zero counters");
            }
            if ((e = hipStreamSynchronize(x.stream())) != hipSuccess) return x.eng->hipfail(e, "sync");
            return fork_point(x);
        });
    }
    // where the next memquota replay forks from the main stream (after the counters were last read)
    int fork_point(Member& x) {
        if (!x.fork) return MXP_OK;  // (mxp_group_create: the events come next)
        const hipError_t e = hipEventRecord(x.fork, x.stream());
        return e == hipSuccess ? MXP_OK : x.eng->hipfail(e, "quota fork point");
    }
    long long* totals(Member& x) const {
        return (long long*)(reduce == MXP_REDUCE_NONE ? x.step.p : x.total.p);
    }
    // the main stream of every member joins its pending quota replay
    int join_quota(Member& x) {
        if (!x.q_pending) return MXP_OK;
        hipError_t e = hipStreamWaitEvent(x.stream(), x.join, 0);
        if (e != hipSuccess) return x.eng->hipfail(e, "join quota stream");
        x.q_pending = false;
        return MXP_OK;
    }
    // the shard layout of a batch call
    void set_bounds(const std::vector<uint64_t>& counts) {
        lo.assign(size() + 1, 0);
        for (uint32_t k = 0; k < size(); k++) lo[k + 1] = lo[k] + counts[k];
    }
    // copy member 0's vocabulary (names in position order, types) into member k (appending the
    // names it lacks: positions stay identical, nothing compiled is reset)
    void sync_vocab(uint32_t k) {
        mxp_engine* a = m[0].eng;
        mxp_engine* b = m[k].eng;
        for (size_t i = b->vocab_names.size(); i < a->vocab_names.size(); i++) {
            const std::string& nm = a->vocab_names[i];
            b->vocab[nm] = a->vocab[nm];
            b->vocab_index[nm] = (uint32_t)i;
            b->vocab_names.push_back(nm);
        }
    }
};

struct mxp_gbatch {
    std::vector<mxp_dbatch*> db;
    std::vector<uint32_t> n;
};

struct mxp_gquota {
    std::vector<mxp_quota*> q;
    std::vector<uint32_t> owner;
    uint32_t n_keys = 0;
};

struct mxp_gqbatch {
    struct Part {
        DevBuf key, amount, be, granted;
        std::vector<uint32_t> pos;  // positions of the part's requests in the caller's order
        PinnedVec<uint32_t> hkey;
        PinnedVec<int64_t> hamount, hgranted;
        PinnedVec<uint8_t> hbe;
    };
    Fixed<Part> part;
    uint32_t n = 0;
    bool evaluated = false;
};

struct mxp_glist {
    std::vector<mxp_list*> l;
};

namespace {

// member k's contiguous view of one host batch: columns offset by the shard's first request, the
// string / time / map tables shared
struct SplitView {
    std::vector<mxp_bag_batch> b;
    std::vector<std::vector<const uint8_t*>> kinds;
    std::vector<std::vector<const uint64_t*>> values;
    std::vector<const mxp_bag_batch*> ptrs;
    SplitView(const mxp_bag_batch* src, uint32_t n) : b(n), kinds(n), values(n), ptrs(n) {
        for (uint32_t k = 0; k < n; k++) {
            uint64_t lo, hi;
            mxp_group_shard_bounds(src->n_requests, k, n, &lo, &hi);
            b[k] = *src;
            b[k].n_requests = (uint32_t)(hi - lo);
            kinds[k].resize(src->n_columns);
            values[k].resize(src->n_columns);
            for (uint32_t c = 0; c < src->n_columns; c++) {
                kinds[k][c] = src->kinds && src->kinds[c] ? src->kinds[c] + lo : nullptr;
                values[k][c] = src->values && src->values[c] ? src->values[c] + lo : nullptr;
            }
            b[k].kinds = src->n_columns ? kinds[k].data() : src->kinds;
            b[k].values = src->n_columns ? values[k].data() : src->values;
            ptrs[k] = &b[k];
        }
    }
};

}  // namespace

// (resolver.cpp) a member's finish with the group's placement, and dropping a submitted job
int mxp_resolve_finish_placed(mxp_resolve_job* job, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off,
                              void* sel_rules, const mxp_resolve_place& place, uint64_t first_cap = 0);
void mxp_resolve_job_free(mxp_resolve_job* job);

extern "C" {

void mxp_group_shard_bounds(uint64_t n_total, uint32_t member, uint32_t n_members, uint64_t* lo, uint64_t* hi) {
    if (!n_members) n_members = 1;
    const uint64_t base = n_total / n_members, extra = n_total % n_members;
    const uint64_t a = (uint64_t)member * base + std::min<uint64_t>(member, extra);
    if (lo) *lo = a;
    if (hi) *hi = a + base + (member < extra ? 1 : 0);
}

int mxp_group_key_owners(const double* weights, uint32_t n_keys, uint32_t n_members, uint32_t* owner) {
    if ((n_keys && (!weights || !owner)) || !n_members) return MXP_ERR_ARG;
    std::vector<uint32_t> order(n_keys);
    for (uint32_t i = 0; i < n_keys; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return weights[a] > weights[b]; });
    // min-heap of (load, member)
    std::vector<std::pair<double, uint32_t>> heap;
    for (uint32_t r = 0; r < n_members; r++) heap.push_back({0.0, r});
    auto cmp = [](const std::pair<double, uint32_t>& a, const std::pair<double, uint32_t>& b) { return a > b; };
    std::make_heap(heap.begin(), heap.end(), cmp);
    for (uint32_t k : order) {
        std::pop_heap(heap.begin(), heap.end(), cmp);
        auto& top = heap.back();
        owner[k] = top.second;
        top.first += weights[k];
        std::push_heap(heap.begin(), heap.end(), cmp);
    }
    return MXP_OK;
}

static std::string g_create_error;  // (mxp_group_last_error(NULL): why the last create failed)

int mxp_group_create(const int* devices, uint32_t n, uint32_t flags, mxp_group** out) {
    if (!out) return MXP_ERR_ARG;
    *out = nullptr;
    if (!devices || !n || (flags & ~(MXP_GROUP_HOST_REDUCE | MXP_GROUP_RCCL_SINGLE))) {
        g_create_error = "mxp_group_create: bad arguments";
        return MXP_ERR_ARG;
    }
    DeviceGuard guard;
    std::unique_ptr<mxp_group> g(new (std::nothrow) mxp_group());
    if (!g) return MXP_ERR_NOMEM;
    g->m.resize(n);
    for (uint32_t k = 0; k < n; k++) {
        if (devices[k] < 0) {
            g_create_error = "mxp_group_create: device " + std::to_string(devices[k]) + " (groups need GPUs)";
            for (uint32_t j = 0; j < k; j++) mxp_engine_destroy(g->m[j].eng);
            return MXP_ERR_ARG;
        }
        g->m[k].device = devices[k];
        const int rc = mxp_engine_create(devices[k], &g->m[k].eng);
        if (rc) {
            g_create_error = "mxp_group_create: engine on device " + std::to_string(devices[k]) + " failed";
            for (uint32_t j = 0; j < k; j++) mxp_engine_destroy(g->m[j].eng);
            return rc;
        }
    }
    g->crew.reset(new Crew(n));
    // the reduction: RCCL over distinct devices, else the host
    bool distinct = true;
    for (uint32_t a = 0; a < n; a++)
        for (uint32_t b = a + 1; b < n; b++) distinct &= devices[a] != devices[b];
    const bool want_rccl = (n > 1 || (flags & MXP_GROUP_RCCL_SINGLE)) && !(flags & MXP_GROUP_HOST_REDUCE);
    g->reduce = n > 1 || (flags & (MXP_GROUP_RCCL_SINGLE | MXP_GROUP_HOST_REDUCE)) ? MXP_REDUCE_HOST : MXP_REDUCE_NONE;
    if (want_rccl && !distinct) {
        g->last_error = "reduction on the host: a device appears twice in the group (RCCL needs one rank per GPU)";
    } else if (want_rccl) {
        std::lock_guard<std::mutex> lk(g_rccl_mu);
        Rccl& R = rccl();
        if (!R.load()) {
            g->last_error = "reduction on the host: " + R.err;
        } else {
            std::vector<ncclComm_t> comms(n, nullptr);
            const ncclResult_t r = R.CommInitAll(comms.data(), (int)n, devices);
            if (r != ncclSuccess) {
                g->last_error = "reduction on the host: ncclCommInitAll: " + R.text(r);
            } else {
                for (uint32_t k = 0; k < n; k++) g->m[k].comm = comms[k];
                g->reduce = MXP_REDUCE_RCCL;
            }
        }
    }
    for (uint32_t k = 0; k < n; k++) {
        auto& x = g->m[k];
        hipError_t e;
        if ((e = hipSetDevice(x.device)) != hipSuccess || (e = hipEventCreateWithFlags(&x.fork, kOrderEvent)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&x.join, kOrderEvent)) != hipSuccess ||
            (e = hipStreamCreateWithFlags(&x.es, hipStreamNonBlocking)) != hipSuccess) {
            if (e != hipSuccess) x.es = nullptr;
            g_create_error = std::string("mxp_group_create: events / stream: ") + hipGetErrorString(e);
            mxp_group_destroy(g.release());
            return MXP_ERR_DEVICE;
        }
    }
    if (int rc = g->reset_counters()) {
        g_create_error = g->last_error;
        mxp_group_destroy(g.release());
        return rc;
    }
    *out = g.release();
    return MXP_OK;
}

void mxp_group_destroy(mxp_group* g) {
    if (!g) return;
    DeviceGuard guard;
    for (auto& x : g->m) {
        if (!x.eng) continue;
        (void)hipSetDevice(x.device);
        if (x.q_pending) (void)hipEventSynchronize(x.join);
        (void)hipStreamSynchronize(x.stream());
        (void)hipStreamSynchronize(x.eng->stream);
    }
    if (g->reduce == MXP_REDUCE_RCCL) {
        std::lock_guard<std::mutex> lk(g_rccl_mu);
        for (auto& x : g->m)
            if (x.comm) (void)rccl().CommDestroy(x.comm);
    }
    g->crew.reset();
    for (auto& x : g->m) {
        if (!x.eng) continue;
        (void)hipSetDevice(x.device);
        x.step.reset();
        x.total.reset();
        x.match.reset();
        x.err.reset();
        x.req_err.reset();
        if (x.qs) (void)hipStreamDestroy(x.qs);
        if (x.es) (void)hipStreamDestroy(x.es);
        if (x.fork) (void)hipEventDestroy(x.fork);
        if (x.join) (void)hipEventDestroy(x.join);
        mxp_engine_destroy(x.eng);
        x.eng = nullptr;
    }
    delete g;
}

const char* mxp_group_last_error(const mxp_group* g) { return g ? g->last_error.c_str() : g_create_error.c_str(); }
uint32_t mxp_group_size(const mxp_group* g) { return g ? g->size() : 0; }
int mxp_group_reduce_mode(const mxp_group* g) { return g ? g->reduce : -1; }

mxp_engine* mxp_group_engine(mxp_group* g, uint32_t member) {
    return g && member < g->size() ? g->m[member].eng : nullptr;
}

void* mxp_group_stream(mxp_group* g, uint32_t member) {
    return g && member < g->size() ? (void*)g->m[member].stream() : nullptr;
}

int mxp_group_locate(const mxp_group* g, uint64_t request, uint32_t* member, uint32_t* local) {
    if (!g || g->lo.empty() || request >= g->lo.back()) return MXP_ERR_ARG;
    const uint32_t k = (uint32_t)(std::upper_bound(g->lo.begin(), g->lo.end(), request) - g->lo.begin()) - 1;
    if (member) *member = k;
    if (local) *local = (uint32_t)(request - g->lo[k]);
    return MXP_OK;
}

// ------------------------------------------------------------------------------ configuration
int mxp_group_vocab_set(mxp_group* g, const char* const* names, const int32_t* value_types, uint32_t n) {
    if (!g) return MXP_ERR_ARG;
    DeviceGuard guard;
    g->finder = false;
    return g->each([&](uint32_t k) { return mxp_vocab_set(g->m[k].eng, names, value_types, n); });
}

int mxp_group_vocab_set_finder(mxp_group* g, mxp_attr_finder find, void* ctx) {
    if (!g || !find) return MXP_ERR_ARG;
    DeviceGuard guard;
    g->finder = true;
    return g->each([&](uint32_t k) {
        return k == 0 ? mxp_vocab_set_finder(g->m[0].eng, find, ctx) : mxp_vocab_set(g->m[k].eng, nullptr, nullptr, 0);
    });
}

int mxp_group_ruleset_compile(mxp_group* g, const char* const* exprs, uint32_t n, int32_t* status) {
    if (!g || (n && !exprs)) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::vector<std::vector<int32_t>> st(g->size(), std::vector<int32_t>(n, 0));
    int rc;
    if (g->finder) {
        // member 0 first (the finder is asked on this thread), the others with its vocabulary
        if ((rc = g->each([&](uint32_t k) { return k == 0 ? mxp_ruleset_compile(g->m[0].eng, exprs, n, st[0].data()) : 0; })))
            return rc;
        rc = g->each([&](uint32_t k) {
            if (k == 0) return 0;
            g->sync_vocab(k);
            return mxp_ruleset_compile(g->m[k].eng, exprs, n, st[k].data());
        });
    } else {
        rc = g->each([&](uint32_t k) { return mxp_ruleset_compile(g->m[k].eng, exprs, n, st[k].data()); });
    }
    if (rc) return rc;
    for (uint32_t k = 1; k < g->size(); k++)
        if (st[k] != st[0]) return g->fail(MXP_ERR_STATE, "members compiled the rule set differently");
    if (status && n) memcpy(status, st[0].data(), (size_t)n * 4);
    g->R = n;
    return g->reset_counters();
}

int mxp_group_resolver_set(mxp_group* g, const char* identity_attr, const char* default_ns, const char* const* rule_ns,
                           const uint32_t* variety_mask, const uint8_t* is_tcp, const uint8_t* empty_match, uint32_t n) {
    if (!g) return MXP_ERR_ARG;
    DeviceGuard guard;
    // (member 0 first: with a finder it may give the identity attribute a vocabulary position)
    int rc = g->each([&](uint32_t k) {
        return k == 0 ? mxp_resolver_set(g->m[0].eng, identity_attr, default_ns, rule_ns, variety_mask, is_tcp, empty_match, n)
                      : 0;
    });
    if (rc) return rc;
    return g->each([&](uint32_t k) {
        if (k == 0) return 0;
        if (g->finder) g->sync_vocab(k);
        return mxp_resolver_set(g->m[k].eng, identity_attr, default_ns, rule_ns, variety_mask, is_tcp, empty_match, n);
    });
}

// ------------------------------------------------------------------------------ device-resident shards
int mxp_group_upload(mxp_group* g, const mxp_bag_batch* const* shards, uint32_t n_shards, uint32_t flags,
                     mxp_gbatch** out) {
    if (!g || !shards || !out || n_shards != g->size()) return MXP_ERR_ARG;
    for (uint32_t k = 0; k < n_shards; k++)
        if (!shards[k]) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::unique_ptr<mxp_gbatch> gb(new mxp_gbatch());
    gb->db.assign(n_shards, nullptr);
    gb->n.assign(n_shards, 0);
    int rc = g->each([&](uint32_t k) {
        gb->n[k] = shards[k]->n_requests;
        return mxp_batch_upload_ex(g->m[k].eng, shards[k], flags, &gb->db[k]);
    });
    if (rc) {
        mxp_group_batch_free(g, gb.release());
        return rc;
    }
    std::vector<uint64_t> cnt(gb->n.begin(), gb->n.end());
    g->set_bounds(cnt);
    *out = gb.release();
    return MXP_OK;
}

int mxp_group_upload2(mxp_group* g, const mxp_bag_batch2* const* shards, uint32_t n_shards, uint32_t flags,
                      mxp_gbatch** out) {
    if (!g || !shards || !out || n_shards != g->size()) return MXP_ERR_ARG;
    for (uint32_t k = 0; k < n_shards; k++)
        if (!shards[k]) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::unique_ptr<mxp_gbatch> gb(new mxp_gbatch());
    gb->db.assign(n_shards, nullptr);
    gb->n.assign(n_shards, 0);
    int rc = g->each([&](uint32_t k) {
        gb->n[k] = shards[k]->base.n_requests;
        return mxp_batch_upload2(g->m[k].eng, shards[k], flags, &gb->db[k]);
    });
    if (rc) {
        mxp_group_batch_free(g, gb.release());
        return rc;
    }
    std::vector<uint64_t> cnt(gb->n.begin(), gb->n.end());
    g->set_bounds(cnt);
    *out = gb.release();
    return MXP_OK;
}

int mxp_group_upload_split(mxp_group* g, const mxp_bag_batch* batch, uint32_t flags, mxp_gbatch** out) {
    if (!g || !batch) return MXP_ERR_ARG;
    SplitView v(batch, g->size());
    return mxp_group_upload(g, v.ptrs.data(), g->size(), flags, out);
}

int mxp_group_batch_wait_copied(mxp_gbatch* gb) {
    if (!gb) return MXP_ERR_ARG;
    for (mxp_dbatch* db : gb->db)
        if (db && mxp_batch_wait_copied(db)) return MXP_ERR_DEVICE;
    return MXP_OK;
}

void mxp_group_batch_free(mxp_group* g, mxp_gbatch* gb) {
    if (!gb) return;
    DeviceGuard guard;
    for (uint32_t k = 0; g && k < gb->db.size() && k < g->size(); k++)
        if (gb->db[k]) mxp_batch_free(g->m[k].eng, gb->db[k]);
    delete gb;
}

uint32_t mxp_group_batch_requests(const mxp_gbatch* gb, uint32_t member) {
    return gb && member < gb->n.size() ? gb->n[member] : 0;
}

int mxp_group_eval(mxp_group* g, mxp_gbatch* gb, uint32_t flags) {
    if (!g || !gb || gb->db.size() != g->size() || (flags & ~MXP_GROUP_EVAL_ERR_BITMAP)) return MXP_ERR_ARG;
    if (!g->m[0].eng->have_rules) return g->fail(MXP_ERR_STATE, "no rule set compiled");
    const bool bitmap = (flags & MXP_GROUP_EVAL_ERR_BITMAP) != 0;
    const size_t W = (g->R + 31) / 32;
    DeviceGuard guard;
    std::vector<uint64_t> cnt(gb->n.begin(), gb->n.end());
    g->set_bounds(cnt);
    return g->each([&](uint32_t k) -> int {
        auto& x = g->m[k];
        const uint32_t n = gb->n[k];
        x.eval_n = n;
        x.eval_bitmap = bitmap;
        x.evaluated = true;
        if (!n) return MXP_OK;
        hipError_t e;
        if ((e = x.match.reserve(W * n * 4)) != hipSuccess) return x.eng->hipfail(e, "alloc match bitmap");
        unsigned long long* hits = (unsigned long long*)x.step.p;
        if (bitmap) {
            if ((e = x.err.reserve(W * n * 4)) != hipSuccess) return x.eng->hipfail(e, "alloc error bitmap");
            return mxp_batch_eval_device_hits(x.eng, gb->db[k], x.stream(), x.match.as<uint32_t>(), x.err.as<uint32_t>(), hits);
        }
        if ((e = x.req_err.reserve(n)) != hipSuccess) return x.eng->hipfail(e, "alloc request errors");
        return mxp_batch_eval_device_compact(x.eng, gb->db[k], x.stream(), x.match.as<uint32_t>(), x.req_err.as<uint8_t>(),
                                             hits);
    });
}

int mxp_group_download(mxp_group* g, uint32_t member, uint32_t* match_bits, uint32_t* err_bits, uint8_t* req_err) {
    if (!g || member >= g->size()) return MXP_ERR_ARG;
    auto& x = g->m[member];
    if (!x.evaluated) return g->fail(MXP_ERR_STATE, "member not evaluated");
    if ((err_bits && !x.eval_bitmap) || (req_err && x.eval_bitmap))
        return g->fail(MXP_ERR_STATE, "the last evaluation wrote the other error form");
    DeviceGuard guard;
    hipError_t e;
    if ((e = hipSetDevice(x.device)) != hipSuccess) return g->hipfail(e, "hipSetDevice");
    if ((e = hipStreamSynchronize(x.stream())) != hipSuccess) return g->hipfail(e, "sync");
    const size_t W = (g->R + 31) / 32, n = x.eval_n;
    if (!n) return MXP_OK;
    if (match_bits && (e = hipMemcpy(match_bits, x.match.p, W * n * 4, hipMemcpyDeviceToHost)) != hipSuccess)
        return g->hipfail(e, "download match");
    if (err_bits && (e = hipMemcpy(err_bits, x.err.p, W * n * 4, hipMemcpyDeviceToHost)) != hipSuccess)
        return g->hipfail(e, "download errors");
    if (req_err && (e = hipMemcpy(req_err, x.req_err.p, n, hipMemcpyDeviceToHost)) != hipSuccess)
        return g->hipfail(e, "download request errors");
    return MXP_OK;
}

// ------------------------------------------------------------------------------ counters
int mxp_group_reduce(mxp_group* g) {
    if (!g) return MXP_ERR_ARG;
    DeviceGuard guard;
    const uint32_t N = std::max<uint32_t>(1, g->R + g->K);
    int rc = g->each([&](uint32_t k) { return g->join_quota(g->m[k]); });
    if (rc) return rc;
    if (g->reduce == MXP_REDUCE_NONE)  // (one member: the counters are the totals)
        return g->each([&](uint32_t k) { return g->fork_point(g->m[k]); });
    if (g->reduce == MXP_REDUCE_RCCL) {
        std::lock_guard<std::mutex> lk(g_rccl_mu);
        Rccl& R = rccl();
        ncclResult_t r = R.GroupStart();
        for (uint32_t k = 0; r == ncclSuccess && k < g->size(); k++) {
            auto& x = g->m[k];
            r = R.AllReduce(x.step.p, x.step.p, N, ncclInt64, ncclSum, x.comm, x.stream());
        }
        const ncclResult_t r2 = R.GroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess) return g->fail(MXP_ERR_DEVICE, "ncclAllReduce: " + R.text(r ? r : r2));
    } else {
        // host: every member's step counters down, summed, the sum back up (synchronous)
        rc = g->each([&](uint32_t k) -> int {
            auto& x = g->m[k];
            x.host_ctr.resize(N);
            hipError_t e;
            if ((e = hipMemcpyAsync(x.host_ctr.data(), x.step.p, (size_t)N * 8, hipMemcpyDeviceToHost, x.stream())) != hipSuccess ||
                (e = hipStreamSynchronize(x.stream())) != hipSuccess)
                return x.eng->hipfail(e, "download step counters");
            return MXP_OK;
        });
        if (rc) return rc;
        g->host_sum.assign(N, 0);
        for (auto& x : g->m)
            for (uint32_t i = 0; i < N; i++) g->host_sum[i] += x.host_ctr[i];
        rc = g->each([&](uint32_t k) -> int {
            auto& x = g->m[k];
            hipError_t e;
            if ((e = hipMemcpyAsync(x.step.p, g->host_sum.data(), (size_t)N * 8, hipMemcpyHostToDevice, x.stream())) != hipSuccess ||
                (e = hipStreamSynchronize(x.stream())) != hipSuccess)
                return x.eng->hipfail(e, "upload summed counters");
            return MXP_OK;
        });
        if (rc) return rc;
    }
    return g->each([&](uint32_t k) -> int {
        auto& x = g->m[k];
        hipError_t e = mxp_launch_group_fold(x.total.as<long long>(), x.step.as<long long>(), N, x.stream());
        return e == hipSuccess ? g->fork_point(x) : x.eng->hipfail(e, "launch counter fold");
    });
}

int mxp_group_counters(mxp_group* g, uint64_t* hits, int64_t* quota_delta) {
    if (!g) return MXP_ERR_ARG;
    DeviceGuard guard;
    auto& x = g->m[0];
    hipError_t e;
    if ((e = hipSetDevice(x.device)) != hipSuccess) return g->hipfail(e, "hipSetDevice");
    if (x.q_pending && (e = hipEventSynchronize(x.join)) != hipSuccess) return g->hipfail(e, "quota sync");
    if ((e = hipStreamSynchronize(x.stream())) != hipSuccess) return g->hipfail(e, "sync");
    const long long* t = g->totals(x);
    if (hits && g->R && (e = hipMemcpy(hits, t, (size_t)g->R * 8, hipMemcpyDeviceToHost)) != hipSuccess)
        return g->hipfail(e, "download hits");
    if (quota_delta && g->K && (e = hipMemcpy(quota_delta, t + g->R, (size_t)g->K * 8, hipMemcpyDeviceToHost)) != hipSuccess)
        return g->hipfail(e, "download quota deltas");
    return MXP_OK;
}

int mxp_group_counters_reset(mxp_group* g) {
    if (!g) return MXP_ERR_ARG;
    DeviceGuard guard;
    return g->reset_counters();
}

int mxp_group_sync(mxp_group* g) {
    if (!g) return MXP_ERR_ARG;
    DeviceGuard guard;
    return g->each([&](uint32_t k) -> int {
        auto& x = g->m[k];
        hipError_t e;
        if (x.q_pending && (e = hipEventSynchronize(x.join)) != hipSuccess) return x.eng->hipfail(e, "quota sync");
        if ((e = hipStreamSynchronize(x.stream())) != hipSuccess) return x.eng->hipfail(e, "sync");
        return MXP_OK;
    });
}

// ------------------------------------------------------------------------------ memquota
int mxp_group_quota_create(mxp_group* g, uint32_t n_keys, const int64_t* max_amount, const int64_t* valid_duration_ns,
                           const uint32_t* owner, mxp_gquota** out) {
    if (!g || !out || (n_keys && (!max_amount || !valid_duration_ns))) return MXP_ERR_ARG;
    for (uint32_t k = 0; owner && k < n_keys; k++)
        if (owner[k] >= g->size()) return g->fail(MXP_ERR_ARG, "quota key owner out of range");
    DeviceGuard guard;
    std::unique_ptr<mxp_gquota> q(new mxp_gquota());
    q->n_keys = n_keys;
    q->q.assign(g->size(), nullptr);
    q->owner.resize(n_keys);
    for (uint32_t k = 0; k < n_keys; k++) q->owner[k] = owner ? owner[k] : k % g->size();
    int rc = g->each([&](uint32_t k) { return mxp_quota_create(g->m[k].eng, n_keys, max_amount, valid_duration_ns, &q->q[k]); });
    if (rc) {
        mxp_group_quota_destroy(g, q.release());
        return rc;
    }
    g->K = n_keys;
    if ((rc = g->reset_counters())) {
        mxp_group_quota_destroy(g, q.release());
        return rc;
    }
    *out = q.release();
    return MXP_OK;
}

void mxp_group_quota_destroy(mxp_group* g, mxp_gquota* q) {
    if (!q) return;
    DeviceGuard guard;
    for (uint32_t k = 0; g && k < q->q.size() && k < g->size(); k++) {
        auto& x = g->m[k];
        (void)hipSetDevice(x.device);
        if (x.q_pending) {
            (void)hipEventSynchronize(x.join);
            x.q_pending = false;
        }
        if (q->q[k]) mxp_quota_destroy(x.eng, q->q[k]);
    }
    delete q;
}

int mxp_group_quota_upload(mxp_group* g, mxp_gquota* q, uint32_t n, const uint32_t* key, const int64_t* amount,
                           const uint8_t* best_effort, mxp_gqbatch** out) {
    if (!g || !q || !out || (n && (!key || !amount || !best_effort)) || q->q.size() != g->size()) return MXP_ERR_ARG;
    for (uint32_t i = 0; i < n; i++)
        if (key[i] >= q->n_keys) return g->fail(MXP_ERR_ARG, "quota key id out of range");
    DeviceGuard guard;
    std::unique_ptr<mxp_gqbatch> qb(new mxp_gqbatch());
    qb->n = n;
    qb->part.resize(g->size());
    const uint32_t* own = q->owner.data();
    int rc = g->each([&](uint32_t k) -> int {
        auto& P = qb->part[k];
        auto& x = g->m[k];
        // this owner's requests, in arrival order (each member scans the stream for its own keys)
        for (uint32_t i = 0; i < n; i++)
            if (own[key[i]] == k) P.pos.push_back(i);
        const size_t m = P.pos.size();
        P.hkey.resize(m);
        P.hamount.resize(m);
        P.hbe.resize(m);
        for (size_t j = 0; j < m; j++) {
            const uint32_t i = P.pos[j];
            P.hkey[j] = key[i];
            P.hamount[j] = amount[i];
            P.hbe[j] = best_effort[i];
        }
        hipError_t e;
        if ((e = P.key.alloc(m * 4)) != hipSuccess || (e = P.amount.alloc(m * 8)) != hipSuccess ||
            (e = P.be.alloc(m)) != hipSuccess || (e = P.granted.alloc(m * 8)) != hipSuccess)
            return x.eng->hipfail(e, "alloc quota requests");
        if (m && ((e = hipMemcpyAsync(P.key.p, P.hkey.data(), m * 4, hipMemcpyHostToDevice, x.stream())) != hipSuccess ||
                  (e = hipMemcpyAsync(P.amount.p, P.hamount.data(), m * 8, hipMemcpyHostToDevice, x.stream())) != hipSuccess ||
                  (e = hipMemcpyAsync(P.be.p, P.hbe.data(), m, hipMemcpyHostToDevice, x.stream())) != hipSuccess))
            return x.eng->hipfail(e, "upload quota requests");
        if ((e = hipStreamSynchronize(x.stream())) != hipSuccess) return x.eng->hipfail(e, "sync");
        return MXP_OK;
    });
    if (rc) {
        mxp_group_quota_batch_free(g, qb.release());
        return rc;
    }
    *out = qb.release();
    return MXP_OK;
}

int mxp_group_quota_eval(mxp_group* g, mxp_gquota* q, mxp_gqbatch* qb, int64_t now_ns) {
    if (!g || !q || !qb || qb->part.size() != g->size() || q->q.size() != g->size()) return MXP_ERR_ARG;
    DeviceGuard guard;
    const bool counted = g->K == q->n_keys;  // (the counters carry this table's deltas)
    qb->evaluated = true;
    return g->each([&](uint32_t k) -> int {
        auto& x = g->m[k];
        auto& P = qb->part[k];
        hipError_t e;
        if (!x.qs) {
            int lo = 0, hi = 0;
            (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
            // (the latency-bound replay first: dispatched ahead of the evaluation's workgroups)
            if ((e = hipStreamCreateWithPriority(&x.qs, hipStreamNonBlocking, hi)) != hipSuccess) {
                x.qs = nullptr;
                return x.eng->hipfail(e, "quota stream");
            }
        }
        // forked at the last reduction (or counter reset): after the fold that read and zeroed the
        // step counters, not after this step's evaluation, which the replay overlaps (the two write
        // disjoint counters); joined by the next reduce / sync
        if ((e = hipStreamWaitEvent(x.qs, x.fork, 0)) != hipSuccess) return x.eng->hipfail(e, "fork quota stream");
        const uint32_t m = (uint32_t)P.pos.size();
        int64_t* delta = counted ? (int64_t*)x.step.p + g->R : nullptr;
        if (m) {
            const int rc = mxp_quota_alloc_device(x.eng, q->q[k], m, P.key.as<uint32_t>(), P.amount.as<int64_t>(),
                                                  P.be.as<uint8_t>(), now_ns, x.qs, P.granted.as<int64_t>(), delta);
            if (rc) return rc;
        }
        if ((e = hipEventRecord(x.join, x.qs)) != hipSuccess) return x.eng->hipfail(e, "join quota stream");
        x.q_pending = true;
        return MXP_OK;
    });
}

int mxp_group_quota_granted(mxp_group* g, mxp_gqbatch* qb, int64_t* granted) {
    if (!g || !qb || (qb->n && !granted) || qb->part.size() != g->size()) return MXP_ERR_ARG;
    if (!qb->evaluated) return g->fail(MXP_ERR_STATE, "quota batch not evaluated");
    DeviceGuard guard;
    return g->each([&](uint32_t k) -> int {
        auto& x = g->m[k];
        auto& P = qb->part[k];
        const size_t m = P.pos.size();
        hipError_t e;
        // (the replay's own event, joined or not: the member's stream is non-blocking, so the
        // legacy-stream copy below does not wait for it)
        if ((e = hipEventSynchronize(x.join)) != hipSuccess) return x.eng->hipfail(e, "quota sync");
        if (!m) return MXP_OK;
        P.hgranted.resize(m);
        if ((e = hipMemcpy(P.hgranted.data(), P.granted.p, m * 8, hipMemcpyDeviceToHost)) != hipSuccess)
            return x.eng->hipfail(e, "download granted");
        for (size_t j = 0; j < m; j++) granted[P.pos[j]] = P.hgranted[j];
        return MXP_OK;
    });
}

void mxp_group_quota_batch_free(mxp_group* g, mxp_gqbatch* qb) {
    if (!qb) return;
    DeviceGuard guard;
    for (uint32_t k = 0; g && k < qb->part.size() && k < g->size(); k++) {
        auto& x = g->m[k];
        (void)hipSetDevice(x.device);
        if (qb->evaluated) (void)hipEventSynchronize(x.join);  // (the replay may still read the requests)
        auto& P = qb->part[k];
        P.key.reset();
        P.amount.reset();
        P.be.reset();
        P.granted.reset();
    }
    delete qb;
}

uint32_t mxp_group_quota_batch_requests(const mxp_gqbatch* qb, uint32_t member) {
    return qb && member < qb->part.size() ? (uint32_t)qb->part[member].pos.size() : 0;
}

int mxp_group_quota_alloc(mxp_group* g, mxp_gquota* q, uint32_t n, const uint32_t* key, const int64_t* amount,
                          const uint8_t* best_effort, int64_t now_ns, int64_t* granted) {
    mxp_gqbatch* qb = nullptr;
    int rc = mxp_group_quota_upload(g, q, n, key, amount, best_effort, &qb);
    if (!rc) rc = mxp_group_quota_eval(g, q, qb, now_ns);
    if (!rc) rc = mxp_group_quota_granted(g, qb, granted);
    mxp_group_quota_batch_free(g, qb);
    return rc;
}

// ------------------------------------------------------------------------------ Resolve
// mxp_group_resolve_batch, and over shards uploaded before (gb, taken over) mxp_group_resolve_uploaded
static int group_resolve(mxp_group* g, mxp_gbatch* gb, const mxp_bag_batch* const* shards, uint32_t n_shards,
                         uint32_t variety, uint32_t flags, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off,
                         void* sel_rules, uint64_t sel_cap) {
    std::unique_ptr<mxp_gbatch, std::function<void(mxp_gbatch*)>> own(gb, [g](mxp_gbatch* b) {
        mxp_group_batch_free(g, b);  // (the members' batches not handed to their Resolve)
    });
    // (shards NULL with narrow uploads: the members' host views)
    std::vector<const mxp_bag_batch*> views;
    if (!shards && gb && g && gb->db.size() == g->size()) {
        for (mxp_dbatch* db : gb->db) views.push_back(db && db->wide ? &db->wide->view : nullptr);
        shards = views.data();
    }
    if (!g || !shards || n_shards != g->size() || !status || !err_rule || !sel_off || (sel_cap && !sel_rules) ||
        (flags & ~(uint32_t)MXP_RESOLVE_IDS_U16) || (gb && gb->db.size() != n_shards))
        return MXP_ERR_ARG;
    for (uint32_t k = 0; k < n_shards; k++)
        if (!shards[k] || (gb && gb->n[k] != shards[k]->n_requests)) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::vector<uint64_t> cnt(n_shards);
    for (uint32_t k = 0; k < n_shards; k++) cnt[k] = shards[k]->n_requests;
    g->set_bounds(cnt);
    // Every member resolves its shard straight into the caller's arrays: status / err_rule at its
    // first request, its batch-local offsets at sel_off + lo (the boundary entry each member shares with
    // the next is rewritten below), and its rule ids at the place the members' counts give it -- the
    // members meet once (Rendezvous), when each knows its own count, before downloading the ids.
    struct Rendezvous {
        std::mutex mu;
        std::condition_variable cv;
        uint32_t arrived = 0, n = 0;
        std::vector<uint64_t> total;
        std::vector<bool> in;
        uint64_t sum = 0;
        void arrive(uint32_t k, uint64_t t) {  // (k's count; idempotent per member)
            std::lock_guard<std::mutex> l(mu);
            if (in[k]) return;
            in[k] = true;
            total[k] = t;
            if (++arrived == n) cv.notify_all();
        }
        void wait() {
            std::unique_lock<std::mutex> l(mu);
            cv.wait(l, [&] { return arrived == n; });
        }
    } rv;
    rv.n = n_shards;
    rv.total.assign(n_shards, 0);
    rv.in.assign(n_shards, false);
    std::atomic<bool> failed{false};
    int rc = g->each([&](uint32_t k) -> int {
        const uint64_t lo = g->lo[k];
        const mxp_resolve_place place = [&](uint64_t t) -> int64_t {
            rv.arrive(k, t);
            rv.wait();
            if (failed.load()) return -1;
            uint64_t base = 0, sum = 0;
            for (uint32_t j = 0; j < n_shards; j++) {
                if (j < k) base += rv.total[j];
                sum += rv.total[j];
            }
            return sum <= sel_cap ? (int64_t)base : -1;
        };
        mxp_dbatch* db = nullptr;
        if (gb) std::swap(db, gb->db[k]);  // (taken over by the member's Resolve)
        const int r = mxp_resolve_placed(g->m[k].eng, db, shards[k], variety, flags, status + lo, err_rule + lo,
                                         sel_off + lo, sel_rules, place, k == 0 ? sel_cap : 0);
        if (r && r != MXP_ERR_NOMEM) failed.store(true);
        rv.arrive(k, 0);  // (a member that failed before its count still lets the others go on)
        return r == MXP_ERR_NOMEM ? MXP_OK : r;
    });
    if (rc) return rc;
    uint64_t total = 0;
    std::vector<uint64_t> base(n_shards, 0);
    for (uint32_t k = 0; k < n_shards; k++) {
        base[k] = total;
        total += rv.total[k];
    }
    // the batch-local offsets rebased (member 0's are already global); each member's first entry is
    // its base (the engines leave it alone: it is the previous member's last entry)
    rc = g->each([&](uint32_t k) -> int {
        const uint64_t lo = g->lo[k], n = cnt[k], b = base[k];
        if (!n) return MXP_OK;
        sel_off[lo] = b;
        if (b)
            for (uint64_t i = 1; i < n; i++) sel_off[lo + i] += b;
        return MXP_OK;
    });
    sel_off[g->lo[n_shards]] = total;
    if (rc) return rc;
    return total <= sel_cap ? MXP_OK : MXP_ERR_NOMEM;
}

// ---- the two-call Resolve (mxp_group_resolve_submit / _finish; the member calls: above extern "C")

struct mxp_gresolve {
    std::vector<mxp_resolve_job*> jobs;  // per member (null: its submit failed)
    std::vector<uint64_t> lo;            // the batch's shard bounds (an upload in between moves g->lo)
    std::vector<uint64_t> cnt;
};

int mxp_group_resolve_submit(mxp_group* g, mxp_gbatch* gb, const mxp_bag_batch* const* shards, uint32_t n_shards,
                             uint32_t variety, uint32_t flags, mxp_gresolve** out) {
    std::unique_ptr<mxp_gbatch, std::function<void(mxp_gbatch*)>> own(gb, [g](mxp_gbatch* b) {
        mxp_group_batch_free(g, b);  // (the members' batches not handed to their submit)
    });
    if (!g || !gb || !out || n_shards != g->size() || gb->db.size() != n_shards) return MXP_ERR_ARG;
    for (uint32_t k = 0; k < n_shards; k++)
        if (shards && (!shards[k] || gb->n[k] != shards[k]->n_requests)) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::unique_ptr<mxp_gresolve> r(new mxp_gresolve());
    r->jobs.assign(n_shards, nullptr);
    r->cnt.assign(gb->n.begin(), gb->n.end());
    g->set_bounds(r->cnt);
    r->lo = g->lo;
    int rc = g->each([&](uint32_t k) -> int {
        mxp_dbatch* db = nullptr;
        std::swap(db, gb->db[k]);  // (taken over by the member's submit)
        return mxp_resolve_submit(g->m[k].eng, db, shards ? shards[k] : nullptr, variety, flags, &r->jobs[k]);
    });
    if (rc) {
        for (mxp_resolve_job* j : r->jobs)
            if (j) mxp_resolve_job_free(j);
        return rc;
    }
    *out = r.release();
    return MXP_OK;
}

int mxp_group_resolve_finish(mxp_group* g, mxp_gresolve* r0, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off,
                             void* sel_rules, uint64_t sel_cap) {
    std::unique_ptr<mxp_gresolve> r(r0);
    if (!g || !r || r->jobs.size() != g->size()) {
        if (r)
            for (mxp_resolve_job*& j : r->jobs) mxp_resolve_job_free(j), j = nullptr;
        return MXP_ERR_ARG;
    }
    auto drop = [&] {
        for (mxp_resolve_job*& j : r->jobs)
            if (j) mxp_resolve_job_free(j), j = nullptr;
    };
    if (!status || !err_rule || !sel_off || (sel_cap && !sel_rules)) {
        drop();
        return MXP_ERR_ARG;
    }
    DeviceGuard guard;
    const uint32_t n_shards = g->size();
    g->lo = r->lo;  // (pair errors and locate refer to this batch again)
    // as group_resolve: every member resolves into the caller's arrays, its ids at the base the
    // members agree on once each knows its own count
    std::mutex mu;
    std::condition_variable cv;
    uint32_t arrived = 0;
    std::vector<uint64_t> total_k(n_shards, 0);
    std::vector<bool> in(n_shards, false);
    auto arrive = [&](uint32_t k, uint64_t t) {
        std::lock_guard<std::mutex> l(mu);
        if (in[k]) return;
        in[k] = true;
        total_k[k] = t;
        if (++arrived == n_shards) cv.notify_all();
    };
    std::atomic<bool> failed{false};
    int rc = g->each([&](uint32_t k) -> int {
        const uint64_t lo = r->lo[k];
        const mxp_resolve_place place = [&](uint64_t t) -> int64_t {
            arrive(k, t);
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return arrived == n_shards; });
            }
            if (failed.load()) return -1;
            uint64_t base = 0, sum = 0;
            for (uint32_t j = 0; j < n_shards; j++) {
                if (j < k) base += total_k[j];
                sum += total_k[j];
            }
            return sum <= sel_cap ? (int64_t)base : -1;
        };
        mxp_resolve_job* job = nullptr;
        std::swap(job, r->jobs[k]);
        const int rr = mxp_resolve_finish_placed(job, status + lo, err_rule + lo, sel_off + lo, sel_rules, place,
                                                 k == 0 ? sel_cap : 0);
        if (rr && rr != MXP_ERR_NOMEM) failed.store(true);
        arrive(k, 0);  // (a member that failed before its count still lets the others go on)
        return rr == MXP_ERR_NOMEM ? MXP_OK : rr;
    });
    if (rc) return rc;
    uint64_t total = 0;
    std::vector<uint64_t> base(n_shards, 0);
    for (uint32_t k = 0; k < n_shards; k++) {
        base[k] = total;
        total += total_k[k];
    }
    rc = g->each([&](uint32_t k) -> int {  // (the batch-local offsets rebased, as group_resolve)
        const uint64_t lo = r->lo[k], n = r->cnt[k], b = base[k];
        if (!n) return MXP_OK;
        sel_off[lo] = b;
        if (b)
            for (uint64_t i = 1; i < n; i++) sel_off[lo + i] += b;
        return MXP_OK;
    });
    sel_off[r->lo[n_shards]] = total;
    if (rc) return rc;
    return total <= sel_cap ? MXP_OK : MXP_ERR_NOMEM;
}

int mxp_group_resolve_batch(mxp_group* g, const mxp_bag_batch* const* shards, uint32_t n_shards, uint32_t variety,
                            uint32_t flags, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules,
                            uint64_t sel_cap) {
    return group_resolve(g, nullptr, shards, n_shards, variety, flags, status, err_rule, sel_off, sel_rules, sel_cap);
}

int mxp_group_resolve_uploaded(mxp_group* g, mxp_gbatch* gb, const mxp_bag_batch* const* shards, uint32_t n_shards,
                               uint32_t variety, uint32_t flags, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off,
                               void* sel_rules, uint64_t sel_cap) {
    if (!gb) return MXP_ERR_ARG;
    return group_resolve(g, gb, shards, n_shards, variety, flags, status, err_rule, sel_off, sel_rules, sel_cap);
}

int mxp_group_resolve_split(mxp_group* g, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags, uint8_t* status,
                            uint32_t* err_rule, uint64_t* sel_off, void* sel_rules, uint64_t sel_cap) {
    if (!g || !batch) return MXP_ERR_ARG;
    SplitView v(batch, g->size());
    return mxp_group_resolve_batch(g, v.ptrs.data(), g->size(), variety, flags, status, err_rule, sel_off, sel_rules,
                                   sel_cap);
}

int mxp_group_pair_error(mxp_group* g, uint64_t request, uint32_t rule, char* buf, uint32_t cap) {
    if (!g) return MXP_ERR_ARG;
    uint32_t k, local;
    if (mxp_group_locate(g, request, &k, &local)) return g->fail(MXP_ERR_ARG, "request out of range");
    DeviceGuard guard;
    (void)hipSetDevice(g->m[k].device);
    return mxp_pair_error(g->m[k].eng, local, rule, buf, cap);
}

// ------------------------------------------------------------------------------ lists
int mxp_group_list_create(mxp_group* g, int entry_type, const char* const* entries, const uint32_t* entry_lens,
                          uint32_t n_entries, const char* const* overrides, const uint32_t* override_lens,
                          uint32_t n_overrides, mxp_glist** out) {
    if (!g || !out) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::unique_ptr<mxp_glist> l(new mxp_glist());
    l->l.assign(g->size(), nullptr);
    int rc = g->each([&](uint32_t k) {
        return mxp_list_create(g->m[k].eng, entry_type, entries, entry_lens, n_entries, overrides, override_lens, n_overrides,
                               &l->l[k]);
    });
    if (rc) {
        mxp_group_list_destroy(g, l.release());
        return rc;
    }
    *out = l.release();
    return MXP_OK;
}

void mxp_group_list_destroy(mxp_group* g, mxp_glist* l) {
    if (!l) return;
    DeviceGuard guard;
    for (uint32_t k = 0; g && k < l->l.size() && k < g->size(); k++)
        if (l->l[k]) mxp_list_destroy(g->m[k].eng, l->l[k]);
    delete l;
}

mxp_list* mxp_group_list_member(mxp_glist* l, uint32_t member) {
    return l && member < l->l.size() ? l->l[member] : nullptr;
}

int mxp_group_list_check(mxp_group* g, const mxp_glist* l, int blacklist, const uint8_t* sym_bytes,
                         const uint64_t* sym_offsets, uint32_t n, int32_t* codes) {
    if (!g || !l || l->l.size() != g->size() || (n && (!sym_bytes || !sym_offsets || !codes))) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::vector<uint64_t> cnt(g->size());
    for (uint32_t k = 0; k < g->size(); k++) {
        uint64_t lo, hi;
        mxp_group_shard_bounds(n, k, g->size(), &lo, &hi);
        cnt[k] = hi - lo;
    }
    g->set_bounds(cnt);
    return g->each([&](uint32_t k) -> int {
        const uint64_t lo = g->lo[k], m = cnt[k];
        if (!m) return MXP_OK;
        // the shard's offsets rebased to its first symbol
        std::vector<uint64_t> off(m + 1);
        const uint64_t b = sym_offsets[lo];
        for (uint64_t i = 0; i <= m; i++) off[i] = sym_offsets[lo + i] - b;
        return mxp_list_check(g->m[k].eng, l->l[k], blacklist, sym_bytes + b, off.data(), (uint32_t)m, codes + lo);
    });
}

int mxp_group_list_check_device(mxp_group* g, const mxp_glist* l, int blacklist, const uint8_t* const* d_sym_bytes,
                                const uint64_t* const* d_sym_offsets, const uint32_t* n, int32_t* const* d_codes) {
    if (!g || !l || l->l.size() != g->size() || !d_sym_bytes || !d_sym_offsets || !n || !d_codes) return MXP_ERR_ARG;
    DeviceGuard guard;
    std::vector<uint64_t> cnt(n, n + g->size());
    g->set_bounds(cnt);
    return g->each([&](uint32_t k) {
        return mxp_list_check_device(g->m[k].eng, l->l[k], blacklist, d_sym_bytes[k], d_sym_offsets[k], n[k],
                                     g->m[k].stream(), d_codes[k]);
    });
}

}  // extern "C"
