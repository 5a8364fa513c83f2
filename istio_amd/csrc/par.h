// par.h -- host-side parallel loops and string-view hashing for batch packing (engine.cpp pack).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdlib>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mxp {

inline double now_seconds() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Threads for host loops: OMP_NUM_THREADS / MXP_PACK_THREADS when set (the GPU box exports its
// CPU share there), else the hardware count; at most 64.
inline unsigned pack_threads() {
    static const unsigned n = [] {
        const char* e = getenv("MXP_PACK_THREADS");
        if (!e) e = getenv("OMP_NUM_THREADS");
        long v = e ? atol(e) : 0;
        if (v <= 0) v = (long)std::thread::hardware_concurrency();
        return (unsigned)std::max(1L, std::min(v, 64L));
    }();
    return n;
}

// Persistent host workers for the parallel loops: a par_for used to start its threads per call
// (~10-20 us per std::thread), which the large downloads paid per 32 MB chunk and every packing /
// validation pass per call.  One job at a time; a call made while the pool is busy (another
// engine's thread, or a loop nested inside a job) runs on threads of its own as before.
class Pool {
  public:
    static Pool& get() {
        static Pool* p = new Pool();  // (never destroyed: workers may outlive static destructors)
        return *p;
    }
    // f(t) for t in [0, T): t = 0 on the calling thread; false when the pool is busy
    template <class F>
    bool run(unsigned T, F&& f) {
        if (T <= 1 || tl_inside()) return false;
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        grow(T - 1);
        std::function<void(unsigned)> job = [&f](unsigned t) { f(t); };
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &job;
            want_ = T - 1;
            left_ = T - 1;
            gen_++;
        }
        cv_.notify_all();
        tl_inside() = true;
        f(0u);
        tl_inside() = false;
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [&] { return left_ == 0; });
        job_ = nullptr;
        return true;
    }

  private:
    static bool& tl_inside() {
        static thread_local bool v = false;
        return v;
    }
    void grow(unsigned k) {
        while (workers_ < k) {
            const unsigned id = ++workers_;  // worker id: job index id (1..)
            std::thread([this, id] { loop(id); }).detach();
        }
    }
    void loop(unsigned id) {
        tl_inside() = true;
        uint64_t seen = 0;
        for (;;) {
            std::function<void(unsigned)>* job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (id > want_) continue;
                job = job_;
            }
            (*job)(id);
            std::lock_guard<std::mutex> g(mu_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    std::function<void(unsigned)>* job_ = nullptr;
    uint64_t gen_ = 0;
    unsigned want_ = 0, left_ = 0, workers_ = 0;
};

// f(begin, end, worker) over [0, n) in contiguous slices of at least `grain` items.
template <class F>
void par_for(uint64_t n, uint64_t grain, F&& f) {
    if (n == 0) return;
    const uint64_t T = std::min<uint64_t>(pack_threads(), std::max<uint64_t>(1, n / std::max<uint64_t>(grain, 1)));
    if (T <= 1) {
        f(0, n, 0u);
        return;
    }
    const uint64_t step = (n + T - 1) / T;
    auto slice = [&](unsigned t) {
        const uint64_t a = t * step, b = std::min(n, a + step);
        if (a < b) f(a, b, t);
    };
    if (Pool::get().run((unsigned)T, slice)) return;
    std::vector<std::thread> th;
    th.reserve(T - 1);
    for (uint64_t t = 1; t < T; t++) th.emplace_back([&slice, t] { slice((unsigned)t); });
    slice(0u);
    for (auto& x : th) x.join();
}

// 64-bit hash of a byte string (wyhash-style multiply-fold over 8-byte words)
inline uint64_t hash_bytes(const char* p, size_t n) {
    const uint64_t k0 = 0xa0761d6478bd642full, k1 = 0xe7037ed1a0b428dbull;
    auto mix = [](uint64_t a, uint64_t b) {
        __uint128_t r = (__uint128_t)a * b;
        return (uint64_t)r ^ (uint64_t)(r >> 64);
    };
    uint64_t h = k0 ^ (n * k1);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        __builtin_memcpy(&w, p + i, 8);
        h = mix(h ^ w, k1);
    }
    uint64_t w = 0;
    if (i < n) __builtin_memcpy(&w, p + i, n - i);
    return mix(h ^ w ^ ((uint64_t)(n - i) << 56), k0);
}

struct SvHash {
    size_t operator()(std::string_view s) const noexcept { return (size_t)hash_bytes(s.data(), s.size()); }
};
using SvMap = std::unordered_map<std::string_view, uint32_t, SvHash>;

// rep[i], i in [0, m): the first j <= i with eq(i, j) (keys given by hash(i) and eq).  Equal keys
// have equal hashes, so the items are split into hash shards searched in parallel, each with an
// open-addressing table visited in index order.
template <class H, class E>
void dedupe_first(uint32_t m, H&& hash, E&& eq, std::vector<uint32_t>& rep) {
    rep.resize(m);
    if (m == 0) return;
    const unsigned T = (unsigned)std::min<uint64_t>(pack_threads(), std::max<uint64_t>(1, m / 4096));
    std::vector<uint8_t> shard(m);
    std::vector<std::vector<uint32_t>> items(T);
    for (uint32_t i = 0; i < m; i++) {
        shard[i] = (uint8_t)((hash(i) >> 40) % T);
        items[shard[i]].push_back(i);
    }
    auto run = [&](unsigned t) {
        const std::vector<uint32_t>& it = items[t];
        size_t cap = 16;
        while (cap < 2 * it.size()) cap <<= 1;
        std::vector<uint32_t> tab(cap, ~0u);
        for (uint32_t i : it) {
            const uint64_t h = hash(i);
            size_t k = (size_t)h & (cap - 1);
            for (;; k = (k + 1) & (cap - 1)) {
                const uint32_t j = tab[k];
                if (j == ~0u) {
                    tab[k] = i;
                    rep[i] = i;
                    break;
                }
                if (hash(j) == h && eq(i, j)) {
                    rep[i] = j;
                    break;
                }
            }
        }
    };
    if (Pool::get().run(T, run)) return;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; t++) th.emplace_back(run, t);
    run(0);
    for (auto& x : th) x.join();
}

}  // namespace mxp
