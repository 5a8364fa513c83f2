// engine_impl.h -- engine internals shared by the host sources of libmxp (engine.cpp: rule sets,
// packing, evaluation, C-ABI; resolver.cpp: batched runtime.resolver).  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mxp.h"
#include "goutil.h"
#include "ilgen.h"
#include "kargs.h"
#include "pack_args.h"
#include "lower.h"
#include "regex.h"
#include "par.h"
#include "vmopt.h"

// Events that only order device work (a stream waiting on another, or the host waiting before it
// releases scratch): no system-scope release when recorded.  A default event's record writes back
// and invalidates the caches for host visibility, which the next evaluation then waits out at its
// start (~20 us between back-to-back evaluations, profiles/r4_final kernel trace).
static constexpr unsigned kOrderEvent = hipEventDisableTiming | hipEventDisableSystemFence;

extern "C" hipError_t mxp_launch_eval(const mxp_kargs* args, uint32_t grid_x, uint32_t grid_y, int vm, hipStream_t s);
extern "C" hipError_t mxp_launch_index(const mxp_kargs* args, uint32_t grid, hipStream_t s);
extern "C" hipError_t mxp_launch_d2h_copy(void* dst, const void* src, uint64_t n, hipStream_t s);
extern "C" hipError_t mxp_launch_d2h_copy_ids(void* dst, const void* src, const uint64_t* count, uint32_t isz, uint64_t cap,
                                              hipStream_t s);
extern "C" hipError_t mxp_launch_vtd_final(const mxp_kargs* args, const mxp_vtd_final_args* f, hipStream_t s);
extern "C" hipError_t mxp_launch_heads(const mxp_kargs* args, const uint32_t* cols, uint32_t nrow, uint4* heads, hipStream_t s);
extern "C" hipError_t mxp_launch_inject(const mxp_kargs* args, uint32_t grid, hipStream_t s);
extern "C" hipError_t mxp_launch_fill(const mxp_kargs* args, uint32_t n_fills, hipStream_t s);
extern "C" hipError_t mxp_launch_vtfill(const mxp_kargs* args, uint32_t n_fills, hipStream_t s);
extern "C" hipError_t mxp_launch_dtp_sort(const mxp_kargs* args, hipStream_t s);
extern "C" hipError_t mxp_launch_dtp_hits(const uint32_t* part, uint32_t tiles, uint32_t n_rules,
                                          unsigned long long* hits, hipStream_t s);
extern "C" hipError_t mxp_launch_vt_classify(const mxp_kargs* args, hipStream_t s);
extern "C" hipError_t mxp_launch_vt_lookup(const mxp_kargs* args, hipStream_t s);
extern "C" hipError_t mxp_launch_vt_eval(const mxp_kargs* args, uint32_t tiles, uint32_t wchunks, hipStream_t s);
extern "C" hipError_t mxp_launch_hits(const uint32_t* match, uint32_t n, uint32_t n_rules, uint32_t n_words,
                                      unsigned long long* hits, hipStream_t s, const uint32_t* gate = nullptr,
                                      unsigned long long* stats = nullptr, uint32_t* gate_next = nullptr,
                                      uint32_t force = 0);
extern "C" hipError_t mxp_launch_hits_gate(const unsigned long long* stats, uint32_t n, uint32_t n_words,
                                           uint32_t* gate, uint32_t force, hipStream_t s);


// mxp_resolve_batch_ex for one member of a device group (group.cpp): once the request's selected-rule
// count of the batch is known, place(total) returns the index in the caller's sel_rules where this
// batch's ids go (blocking until every member knows its count), or -1 when the whole list does not
// fit; the ids are then downloaded straight there.  sel_off gets the batch-local offsets.
using mxp_resolve_place = std::function<int64_t(uint64_t)>;
// db (nullable): the batch, uploaded before and taken over by the call (mxp_resolve_uploaded)
// first_cap: the whole list's capacity when this member's ids go first (member 0; 0: not first)
int mxp_resolve_placed(mxp_engine* eng, mxp_dbatch* db, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                       uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules,
                       const mxp_resolve_place& place, uint64_t first_cap = 0);

// Device blocks of freed batches, reused by later uploads (mxp_batch_free hands a batch's blocks to
// its engine's bin with events recorded on every stream that read the batch; mxp_batch_upload draws
// from it).  A hipFree synchronises the whole device -- ~0.2 ms each, ~25 per batch, so freeing one
// batch stalled a fresh-batch step behind every kernel in flight; a drawn block waits only for the
// events of the batch it came from (long complete in a steady upload / evaluate / free loop).
struct BlockBin {
    struct Group {
        std::vector<hipEvent_t> evs;  // completion of the work that read the freed batch
        std::vector<std::pair<void*, size_t>> blks;
        bool done = false;
    };
    std::vector<Group> groups;  // oldest first
    size_t bytes = 0;
    // at most this many bytes kept (beyond: the oldest groups are freed): MXP_BIN_CAP_MB, else
    // min(8 GiB, 1/16 of the device's memory)
    size_t cap_bytes = 8ull << 30;
    bool cap_set = false;
    std::mutex mu;  // (a failed hipMalloc on any thread may drain every engine's bin: bins_release_all)
    BlockBin();
    ~BlockBin();
    bool take(size_t want, void** p, size_t* cap);
    void put(Group&& g);
    void release();  // every block freed (engine teardown, or a device allocation that failed)
    size_t held();
    size_t cap_locked();  // (with mu held)
};
// every live engine's bin, drained by DevBuf::alloc when hipMalloc runs out of device memory; true
// when any block was freed
bool bins_release_all();
// the bin DevBuf::alloc draws from (set for the duration of an upload, together with the batch
// being built: only that batch's own buffers draw from the bin -- engine scratch grown meanwhile
// is allocated plainly) / DevBuf::reset hands blocks to (a batch free); null elsewhere
extern thread_local BlockBin* g_bin_take;
extern thread_local const void* g_bin_db;      // the mxp_dbatch under construction
extern thread_local size_t g_bin_db_size;
extern thread_local std::vector<std::pair<void*, size_t>>* g_bin_give;

// Page-locked host memory for host vectors the device writes into (download() then copies straight
// into them: no bounce, no page faults of fresh pages each batch); elements default-initialised, so
// resize() does not zero what the download overwrites.  Falls back to malloc without a device.
template <class T>
struct PinnedAlloc {
    using value_type = T;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U>&) {}
    T* allocate(size_t n) {
        void* p = nullptr;
        if (hipHostMalloc(&p, n * sizeof(T) + 16, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            p = std::malloc(n * sizeof(T) + 16);
            if (!p) throw std::bad_alloc();
        }
        return (T*)p;
    }
    void deallocate(T* p, size_t) {
        hipPointerAttribute_t pa;
        const bool pinned = hipPointerGetAttributes(&pa, p) == hipSuccess && pa.type == hipMemoryTypeHost;
        (void)hipGetLastError();
        if (pinned) (void)hipHostFree(p);
        else std::free(p);
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new ((void*)p) U;
        else ::new ((void*)p) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const PinnedAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U>&) const { return false; }
};

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;    // bytes asked for
    size_t cap = 0;  // bytes the block holds (>= n: a recycled block may be larger)
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    void swap(DevBuf& o) {  // (two engine buffers trade blocks)
        std::swap(p, o.p);
        std::swap(n, o.n);
        std::swap(cap, o.cap);
    }
    ~DevBuf() { reset(); }
    void reset() {
        if (p) {
            if (g_bin_give) g_bin_give->push_back({p, cap});
            else (void)hipFree(p);
        }
        p = nullptr;
        n = cap = 0;
    }
    bool in_batch() const {
        return g_bin_take && (const char*)this >= (const char*)g_bin_db &&
               (const char*)this < (const char*)g_bin_db + g_bin_db_size;
    }
    hipError_t alloc(size_t bytes) {
        reset();
        if (bytes == 0) bytes = 16;
        n = bytes;
        if (in_batch() && g_bin_take->take(bytes, &p, &cap)) return hipSuccess;
        cap = bytes;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipErrorOutOfMemory && bins_release_all()) {  // idle recycled blocks first
            (void)hipGetLastError();
            e = hipMalloc(&p, bytes);
        }
        if (e != hipSuccess) {
            p = nullptr;
            n = cap = 0;
        }
        return e;
    }
    // grow-only: keeps the allocation when it is large enough (engine-owned scratch reused across calls)
    hipError_t reserve(size_t bytes) {
        if (p && cap >= (bytes ? bytes : 16)) return hipSuccess;
        return alloc(bytes);
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

// Global-memory thread sets of the NFAs wider than the private-memory walk (dfa_dev.h
// mxp_nfa_run_global): slots of MXP_NFA_SLOT_WORDS(wmax) words, one per wavefront walking such an
// NFA, claimed through busy flags; at most 512 MB, between 64 and 2048 slots.
struct NfaScratch {
    DevBuf words, busy;
    uint32_t wmax = 0, nslots = 0;
    int ensure(uint32_t w) {
        if (w <= wmax) return 0;
        const uint64_t slot_bytes = MXP_NFA_SLOT_WORDS(w) * 8ull;
        const uint32_t ns = (uint32_t)std::max<uint64_t>(64, std::min<uint64_t>(2048, (512ull << 20) / slot_bytes));
        if (words.alloc(slot_bytes * ns) != hipSuccess || busy.alloc((size_t)ns * 4) != hipSuccess ||
            hipMemset(busy.p, 0, (size_t)ns * 4) != hipSuccess) {
            wmax = nslots = 0;
            return MXP_ERR_NOMEM;
        }
        wmax = w;
        nslots = ns;
        return 0;
    }
    void set(mxp_dfa_set* S) const {
        S->nfa_scratch = words.as<uint64_t>();
        S->nfa_busy = busy.as<uint32_t>();
        S->nfa_nslots = nslots;
        S->nfa_wmax = wmax;
    }
};

struct TimeKey {
    int64_t s;
    int32_t ns;
    bool operator<(const TimeKey& o) const { return s != o.s ? s < o.s : ns < o.ns; }
};

constexpr uint64_t kNoValue = ~0ull;

// Device string pool: every string starts 8-byte aligned (zero padded), with 16 bytes of slack at
// the end, so the kernels compare strings a u64 word at a time (two aligned loads + funnel shift for
// unaligned operands) without reading past the allocation.  desc[i] = offset << 24 | length.
inline bool string_pool(const std::vector<std::string>& strs, std::vector<uint64_t>* desc, std::string* blob) {
    desc->assign(strs.size(), 0);
    blob->clear();
    for (size_t i = 0; i < strs.size(); i++) {
        if (strs[i].size() >= (1u << 24)) return false;
        (*desc)[i] = ((uint64_t)blob->size() << 24) | strs[i].size();
        blob->append(strs[i]);
        blob->append((8 - blob->size() % 8) % 8, '\0');
    }
    blob->append(16, '\0');
    return true;
}

// column kinds that pass a guard's want class (W_*) or a virtual-column guard (GK_VCOL)
inline uint32_t okset_of(uint32_t kind) {
    switch (kind) {
    case W_S: return 1u << MXP_STRING;
    case W_B: return 1u << MXP_BOOL;
    case W_I: return (1u << MXP_INT64) | (1u << MXP_DURATION);
    case W_D: return 1u << MXP_DOUBLE;
    default: return 1u << VC_VALUE;  // GK_VCOL
    }
}

// Strings packed 8-aligned into one blob, in the device pool layout of string_pool (desc[i] =
// offset << 24 | length; 16 bytes of slack after finish()).
struct StrPool {
    std::string blob;
    std::vector<uint64_t> desc;
    size_t size() const { return desc.size(); }
    std::string_view operator[](size_t i) const {
        return std::string_view(blob.data() + (desc[i] >> 24), (size_t)(desc[i] & 0xFFFFFFu));
    }
    bool push(std::string_view s) {
        if (s.size() >= (1u << 24)) return false;
        desc.push_back(((uint64_t)blob.size() << 24) | s.size());
        blob.append(s.data(), s.size());
        blob.append((8 - blob.size() % 8) % 8, '\0');
        return true;
    }
    void finish() { blob.append(16, '\0'); }
};

// The device packer's inputs and working tables (pack_device.cpp), per batch: a batch's copies can
// run while an earlier batch's packer still reads its own (blocks recycled through the bin).
struct PackScratch {
    DevBuf pk_soff, pk_sbytes, pk_tsec, pk_tnsec, pk_moff, pk_mkey, pk_mval, pk_ck[66], pk_cv[66];  // (+2: resolver columns)
    DevBuf pk_sid, pk_braw, pk_bcan, pk_tid, pk_use, pk_tab[4], pk_scan, pk_scan_blocks, pk_scan_max;
    DevBuf pk_vtd_lkey, pk_vtd_lcr, pk_vtd_ln, pk_vtd_tkey, pk_vtd_tcr, pk_vtd_meta, pk_rx, pk_rxv;
    DevBuf pk_cv32[66], pk_soff32, pk_moff32;  // narrow batches: the u32 arrays as copied (mxp_batch_upload2)
};

// A narrow batch's host view (mxp_batch_upload2).  The upload's own host passes read the narrow
// arrays (check_batch, the packer's sizes); the v1 layout -- u32 values and offsets widened -- is made
// only for a host pass that reads it (run-time pattern collection, the host packer, the Resolve's
// host namespaces): materialize(), from the caller's arrays, which are valid while the call that
// asks runs.  Until then the view's narrow columns and its offsets are NULL.
struct WideView {
    mxp_bag_batch view;
    mxp_bag_batch2 src;  // (shallow: the caller's arrays)
    std::vector<const uint64_t*> vptr;
    std::vector<std::unique_ptr<uint64_t[]>> vals;  // (uninitialised: the widening writes every word)
    std::unique_ptr<uint64_t[]> soff, moff;
    bool full = false;
    void materialize();  // engine.cpp
};

struct mxp_dbatch {
    uint32_t n = 0;
    // value classes (pack_host): candidate slots whose column has few distinct values in this batch,
    // their class table capacities, the device class tables (vt_t: match words, then error words)
    uint32_t vt_mask = 0;
    std::vector<uint32_t> vt_capc;         // per candidate slot (0: inactive)
    std::vector<uint32_t> vt_meta_h;       // kargs.vt_meta of the batch's plan (first launch)
    DevBuf vt_cls, vt_keys, vt_rep, vt_cnt, vt_t, vt_meta, vtf_slow;
    size_t vt_t_words = 0, vt_keys_n = 0;
    DevBuf kinds, vals, bstr_off, bstr, map_off, map_keys, map_vals, ipof, tsof;
    DevBuf heads;                                     // [head columns][n] string heads (kargs.heads)
    uint32_t heads_ncol = 0;                          // rows the heads cover (mxp_engine::head_cols)
    DevBuf rxof, rx_hdr, rx_trans, rx_ascii, rx_hilo, rx_hicls;  // run-time regexp patterns
    bool rx_nfa = false;                              // one of them compiled to a bit-parallel NFA
    uint32_t rx_wmax = 0;                             // the widest one's thread-set words
    StrPool overlay;                                  // batch strings not in the rule set's pool
    StrPool overlay_bytes;                            // batch byte strings not in the rule set's
    std::vector<TimeKey> overlay_times;
    // device-packed batches (pack_device.cpp): batch-local ids name batch items -- strings G + s,
    // byte strings GB + item, canonical GC + item, times GT + item (items: batch strings / times
    // first, then parsed ip() / timestamp() values by string id) -- read back on demand
    bool dev_packed = false;
    // per stream an evaluation of this batch was enqueued on: an event recorded after that
    // evaluation's last kernel (launch), so mxp_batch_free only collects events and never touches a
    // caller stream that may be gone by then
    std::vector<std::pair<hipStream_t, hipEvent_t>> done_ev;
    // device packing (pack_device.cpp): its scratch; events [0] strings copied, [1] everything the
    // caller handed over copied, [2] packed (the packer stream), [3] ready (after finish_pack's
    // dictionary and heads, on the engine stream);
    // pack_pending: the packer's kernels may still run and the value-class sizing, tables,
    // dictionary and heads are still to do (mxp_engine::finish_pack, at the first evaluation)
    PackScratch pk;
    hipEvent_t pk_ev[4] = {nullptr, nullptr, nullptr, nullptr};  // [3]: ready (finish_pack's kernels)
    bool pack_pending = false, pk_vt_on = false;
    uint32_t pk_ncand = 0;
    void wait_packed() const {  // (the packer's results readable from the host)
        if (pk_ev[2]) (void)hipEventSynchronize(pk_ev[2]);
        if (pk_ev[3]) (void)hipEventSynchronize(pk_ev[3]);
    }
    ~mxp_dbatch() {
        for (auto& se : done_ev) (void)hipEventDestroy(se.second);
        for (hipEvent_t ev : pk_ev)
            if (ev) (void)hipEventDestroy(ev);
    }
    int note_done(hipStream_t s);  // record (creating on first use) the completion event of stream s
    std::unique_ptr<WideView> wide;  // uploaded narrow (mxp_batch_upload2): the host view of the batch
    // set by pack_device (the batch's own scratch, pk): the raw identity / context.protocol columns as
    // uploaded (nullptr: absent from the batch), for the Resolve's device namespaces; res_raw = false
    // when the host packer ran or the columns were not uploaded
    bool res_raw = false;
    const uint8_t* res_id_kind = nullptr;
    const uint64_t* res_id_val = nullptr;
    const uint8_t* res_pr_kind = nullptr;
    const uint64_t* res_pr_val = nullptr;
    bool vtd_ready = false;  // the packer's provisional class tables (engine scratch) hold this batch's
    uint32_t ns = 0, nt = 0, G = 0, GB = 0, GC = 0, GT = 0;
    DevBuf pip, pip_ok, pts_sec, pts_nsec, pts_ok, btsec, btnsec;
    size_t overlay_strings() const { return dev_packed ? ns : overlay.size(); }
    bool overlay_string(uint64_t j, std::string* out) const;       // batch-local string j (id - G)
    bool overlay_bytes_at(uint64_t j, std::string* out) const;     // batch-local raw bytes j (id - GB)
    bool overlay_time(uint64_t j, TimeKey* out) const;             // batch-local time j (id - GT)
};

struct mxp_engine : public mxp::LowerTables {
    int device = 0;
    hipStream_t stream = nullptr;
    BlockBin bin;  // freed batches' device blocks (declared first: destroyed last)
    std::string last_error;

    mxp::Vocabulary vocab;
    std::unordered_map<std::string, uint32_t> vocab_index;  // name -> position in mxp_vocab_set order
    std::vector<std::string> vocab_names;                   // position -> name
    // mxp_vocab_set_finder: names resolved through the caller's finder on first use
    mxp_attr_finder finder = nullptr;
    void* finder_ctx = nullptr;
    std::set<std::string> finder_missing;                   // names the finder did not know
    // vocabulary position of `name`, asking the finder the first time (-1: not in the vocabulary)
    int64_t vocab_pos(const std::string& name) {
        auto it = vocab_index.find(name);
        if (it != vocab_index.end()) return it->second;
        if (!finder || finder_missing.count(name)) return -1;
        const int32_t vt = finder(finder_ctx, name.c_str());
        if (vt < 0) {
            finder_missing.insert(name);
            return -1;
        }
        vocab[name] = vt;
        vocab_index[name] = (uint32_t)vocab_names.size();
        vocab_names.push_back(name);
        return (int64_t)vocab_names.size() - 1;
    }
    // ... without asking the finder (evaluation paths: positions never grow after compile /
    // mxp_resolver_set, whatever batches are evaluated)
    int64_t vocab_find(const std::string& name) const {
        auto it = vocab_index.find(name);
        return it == vocab_index.end() ? -1 : (int64_t)it->second;
    }
    mxp::FuncMap fmap = mxp::default_func_map();

    // rule-set-global interning
    std::unordered_map<std::string, uint32_t> gstr_ids;
    std::vector<std::string> gstrs;
    std::unordered_map<std::string, uint32_t> gbytes_ids;   // exact []byte values
    std::vector<std::string> gbytes;
    std::unordered_map<std::string, uint32_t> gcanon_ids;   // their net.IP.Equal classes
    std::vector<std::string> gcanon;
    std::map<TimeKey, uint32_t> gtime_ids;
    std::vector<TimeKey> gtimes;
    std::vector<std::string> cols;
    std::unordered_map<std::string, uint32_t> col_ids;
    std::vector<std::pair<std::string, std::string>> vcols;
    std::map<std::pair<std::string, std::string>, uint32_t> vcol_ids;
    uint32_t empty_sid = 0;

    struct Rule {
        int32_t status = MXP_RULE_OK;
        std::string error;
        int32_t value_type = 0;
        uint8_t il_ret = 0;
        std::string il_text;
        mxp::LoweredRule low;
    };
    std::vector<Rule> rules;
    bool have_rules = false;
    bool need_ipof = false, need_tsof = false, need_strings = false, need_maps = false, need_rxof = false;
    // regexp DFAs of the rule set's constant patterns (device image rx_set; host copies for folding)
    static constexpr uint32_t kRegexStates = 1u << 16;
    std::map<std::string, std::pair<int32_t, std::string>> rx_ids;  // pattern -> (DFA | -1 | -2, error)
    mxp::DfaSetHost rx_set;
    std::vector<mxp::Dfa> rx_dfas;
    // run-time regexp pattern sources (lower.cpp provenance): columns, virtual map[key] columns
    // (indices before the resolve columns are appended), map columns whose every value is a
    // pattern, and rule-set constants merged into a pattern by `|`
    std::set<uint32_t> rx_cols, rx_vcols, rx_mapcols, rx_consts;
    // the packers' view: pattern columns in the batch layout (virtual columns after the C resolve
    // columns)
    std::vector<uint32_t> rx_pattern_cols() const {
        std::vector<uint32_t> v(rx_cols.begin(), rx_cols.end());
        for (uint32_t j : rx_vcols) v.push_back((uint32_t)cols.size() + j);
        return v;
    }
    DevBuf d_rx_hdr, d_rx_trans, d_rx_ascii, d_rx_hilo, d_rx_hicls;
    bool rx_nfa = false;         // some constant pattern compiled to a bit-parallel NFA (kargs.nfa)
    uint32_t rx_wmax = 0;        // the widest such NFA's thread-set words
    NfaScratch nfa_scratch;      // global thread sets of NFAs wider than MXP_NFA_WIDE_WORDS

    // rule-level tables (one per compile): programs + template code, offsets, constants, strings
    DevBuf d_prog, d_rule_off, d_gstr_off, d_gstr, d_rconst;
    std::vector<mxp_vm_ins> prog_h;    // host copies the plans are built from
    std::vector<uint32_t> off_h;
    std::vector<mxp_guard> guards_h;   // leading-atom guards before any plan drops a prefix guard
    // prefix-guarded regexp rules whose DFA after the literal prefix is a few literal keys
    // (regex.h dfa_literal_keys): the prefix index serves them as direct postings, one per key
    // (string id, exact: the subject must END there), with no VM pass
    std::vector<std::vector<std::pair<uint32_t, uint8_t>>> rx_keys_h;
    std::vector<uint32_t> rule_tmpl_h;
    std::vector<mxp_tmpl> tmpls_h;
    uint32_t n_guarded = 0, n_templated = 0;
    // Value classes (mxp_vt_*): rules whose result depends on one column's (kind, string value)
    // only.  Candidate columns (>= kVtMinRules such rules, at most kVtCandMax) get a slot; a batch
    // whose column has few distinct values (pack time) activates the slot, and the plan of that set
    // of slots leaves those rules to the value-class kernels.
    static constexpr uint32_t kVtMinRules = 8, kVtCandMax = 32, kVtMaxClasses = 4096;
    std::vector<uint32_t> vt_cand_col;     // slot -> column
    std::vector<uint8_t> vt_slot_of_rule;  // rule -> slot, 0xFF none
    // The kernels' tables for one set of value-class slots (mask 0: none, built at compile)
    struct Plan {
        uint32_t mask = 0;
        uint32_t n_glean = 0, n_gvm = 0, n_gall = 0, n_gdeep = 0, lean_cc = 0, n_fills = 0, n_gfill = 0;
        uint32_t n_idx = 0, n_indexed = 0, n_composite = 0, n_alias = 0, n_tmpls = 0, n_segs = 0;
        uint32_t n_dense = 0, n_inj = 0;
        bool post_tmpl = false;  // postings carry template codes (kargs.post_tmpl)
        bool tmpl_lite = false;  // no template holds a lookup, virtual column or regexp (kargs.tmpl_lite)
        DevBuf d_guards, d_groups, d_segs, d_gk, d_tmpls, d_rule_tmpl, d_rule_tmpl2, d_alias_off, d_aliases;
        DevBuf d_idx, d_hents, d_hbits, d_postings, d_plens;
        DevBuf d_glean, d_gvm, d_gall;  // group lists: guard-only groups, groups needing the VM, all but deep
        DevBuf d_gdeep;                 // groups with deep rules (MXP_VM_DEEPREG kernels), every mode
        DevBuf d_fills, d_fill_masks;   // chunks of uniform indexed groups (mxp_fill_kernel)
        DevBuf d_vtfills;               // ... those with value-class merge entries (mxp_vtfill_kernel)
        uint32_t n_vtfills = 0;
        DevBuf d_dense_of, d_inj;
        // value classes: active slot a -> column vt_cols[a], words vt_nw[a]; per group merge entries
        std::vector<uint32_t> vt_cols, vt_nw;
        uint32_t vt_max_nw = 0;
        DevBuf d_gvt_off, d_gvt, d_gvt_mask, d_vt_woff, d_vt_words;
        // deferred index pairs (kargs.dtp_*): possible when every group holding an indexed rule is
        // written by the value-class fill (no plain fill chunks, no dense rules); per group its fill
        // chunk << 8 | position in the chunk
        bool dtp_ok = false;
        DevBuf d_dtp_chunk;
    };
    std::map<uint32_t, std::unique_ptr<Plan>> plans;
    int get_plan(uint32_t mask, Plan** out);
    int build_plan(Plan& P);
    const Plan* plan0() const {
        auto it = plans.find(0);
        return it == plans.end() ? nullptr : it->second.get();
    }
    uint32_t groups_per_wave = 16; // MXP_GPW (A/B on C4: 4 6.50 ms, 8 6.55, 16 6.36; C2 flat; profiles/r1_v15_ab_gpw.log)
    // optional per-kernel timing of device evaluations (mxp_set_timing): events around each launch
    bool timing = false;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool ev_index = false;
    // dense canonical rules (mxp_inject_kernel): rule -> id < 64, and per bitmap word the
    // (bit | id << 5) entries of those rules and their aliases, in slots of MXP_INJ_SLOT dwords
    static constexpr size_t kDenseMin = 8;
    DevBuf d_dense_cm;  // [n] per-request dense masks of the current evaluation
    // referenced attributes (mxp_eval_refs, refs.cpp)
    struct RefComposite {
        uint32_t a_col, b_col, k1, rule;  // `A == K1 && B.startsWith(K2) ...`: B is read iff A == K1
    };
    std::vector<RefComposite> ref_comp;
    std::vector<uint32_t> ref_guard;               // [rule] column its guard reads (MXP_VM_DONE: none)
    std::vector<uint32_t> ref_alias_off, ref_aliases;  // duplicate indexed rules (records name the canonical rule)
    std::vector<uint32_t> vcol_key_sid;            // [virtual column] string id of its map key
    bool refs_exact = true;                        // false: a rule the lowering does not support
    bool refs_on = false;                          // launch(): use the *_refs kernels
    DevBuf d_refs, d_refcount;
    uint32_t refcap = 1u << 20;
    struct RefScope {  // mxp_resolve_refs: one Resolve per request (resolver.cpp results)
        const std::vector<uint32_t>* info;  // namespace id | tcp << 31, or MXP_NS_MISSING / MXP_NS_NOTSTRING
        const uint8_t* status;
        const uint32_t* err_rule;
        uint32_t variety;
    };
    int refs_evaluate(const mxp_bag_batch* b, DevBuf& dm, DevBuf& de, std::unique_ptr<mxp_dbatch>& db,
                      std::vector<mxp_ref_rec>& recs);
    int refs_assemble(const mxp_bag_batch* b, const std::vector<mxp_ref_rec>& recs, const RefScope* scope,
                      uint64_t* ref_off, mxp_attr_ref* out, uint64_t cap);
    int eval_refs(const mxp_bag_batch* b, uint32_t* match, uint32_t* err, uint64_t* ref_off, mxp_attr_ref* out,
                  uint64_t cap);
    // pipelined chunks (launch): the guard-index kernel of each request chunk on a side stream
    static constexpr uint32_t kChunksMax = 8;
    uint32_t chunk_min = 1u << 17, chunks_max = 1;  // off by default: measured slower
    hipStream_t side = nullptr;
    hipEvent_t chunk_ev[kChunksMax + 1] = {};
    // deferred-pair request chunks (launch: index + sort of chunk c on the side stream beside the
    // fill of chunk c - 1; MXP_DTP_CHUNKS)
    static constexpr uint32_t kDtpChunksMax = 16;
    uint32_t dtp_chunks = 1;
    hipEvent_t dtp_cev[kDtpChunksMax + 1] = {};
    // MXP_DEBUG_FLAGS, ablation only: 1 no in-wave VM, 2 no guards (results invalid), 8 no guard index,
    // 16 no composite index, 64 no duplicate folding, 128 plain fill stores, 256 no dense injection,
    // 512 index equality-only guards too, 524288 / 1048576 fused / streaming hit counters forced,
    // 2097152 value-class fill chunks gather from global memory (no LDS staging)
    // fill layout (same-box A/B on C2, profiles/r1_v17_ab_fill*.log: span 1 / chunk 32 0.945 ms,
    // span 4 0.832-0.836, span 4 / chunk 16 0.831; spans 3, 5, 6, 8 and chunks 4..1000 no better)
    uint32_t fill_chunk = MXP_FILL_CHUNK;  // MXP_FILL_CHUNK: groups per fill chunk
    uint32_t fill_span = 4;                // MXP_FILL_SPAN: 256-request spans per fill wave (1..8)
    uint32_t debug_flags = 0;
    // guard-index hash tables hold >= 2^(1 + index_sparsity) slots per key (MXP_INDEX_SPARSITY):
    // a lower load factor shortens the probe chains of the many misses (prefix probes at every key
    // length).  Same-box A/B (profiles/r2_v7_ab_sparse_*.log), ms per evaluation for 0 / 1 / 2 / 3:
    // C4 2.216 / 2.188 / 2.178 / 2.178, C2 0.576 / 0.573 / 0.566 / 0.562.  Round 4, with the
    // occupancy bitmaps (profiles/r4_s2{5,6}_ab_*_sparsity.log) for 1 / 2 / 3 / 4 / 5 / 6 / 8: C4
    // 0.823 / 0.795 / 0.793 / 0.771-0.782 / 0.746 / 0.750 / 0.742, C2 flat (0.404-0.413): a miss
    // whose slot bit is set costs an entry-pair load, and C4 misses at ~14 key lengths per request
    uint32_t index_sparsity = 5;
    // Deferred index pairs (launch, kernels.hip mxp_dtp_*; MXP_DTP=0 turns them off): per index wave
    // room for dtp_cap pairs, then an overflow list of dtp_ovf_cap (MXP_DTP_CAP / MXP_DTP_OVF: tests)
    bool dtp = true;
    // (dtp_cap is also the lists' stride: 2080 entries = 65 lines of 128 bytes.  At 2048 -- an 8 KB,
    // power-of-two stride -- the index waves' appends and the sort's four concurrent list reads fall
    // on aliased HBM channels: C4 0.745 -> 0.710 ms, the path-only routes 0.630 -> 0.618 ms with 2080,
    // settings alternated in one process, profiles/r4_s3{3,4,5}_ab_*_dtpcap.log)
    uint32_t dtp_cap = 2080, dtp_ovf_cap = 1u << 22;
    DevBuf d_dtp_ent, d_dtp_n, d_dtp_ovf, d_dtp_ovf_n, d_dtp_slots, d_dtp_qn;
    bool last_dtp = false;  // the last launch deferred its index pairs (mxp_kernel_times [2])
    bool last_dtp_counted = false;  // ... and counted every true pair in its kernels (no streamed counters)
    // pair Resolve (resolver.cpp): the resolver asks (pair_req) that the next evaluation leave the match
    // bitmap unwritten when every word is a plain fill chunk's; last_pairs is where that evaluation
    // filed its deferred pairs (on: it did; its fills stored the bitmap only if *ovf_n, its overflow
    // count, is nonzero)
    bool pair_req = false;
    struct PairView {
        bool on = false;
        const uint32_t* ovf_n = nullptr;
        const uint16_t* slots = nullptr;
        const uint8_t* qn = nullptr;
        const uint32_t* fills = nullptr;
        uint64_t row = 0;
        uint32_t nch = 0;
    } last_pairs;
    static constexpr uint32_t kDtpHist = 16384;  // MXP_DTP_HIST (kernels.hip): rule sets counted by histogram
    DevBuf d_dtp_part;                // [tiles][(R + 1) / 2] per-tile true-pair histograms
    uint32_t dtp_par = 0;   // d_dtp_ovf_n holds two counter sets: this launch's and the next one's
    hipEvent_t dtp_ev = nullptr;      // recorded after each deferred launch (its last kernel)
    hipStream_t dtp_stream = nullptr; // ... on this stream; a launch on another stream waits for it
    bool dtp_pending = false;
    // MXP_TRACE=1: phase times of evaluations / Resolves on stderr (each phase synchronises the
    // stream first, so traced calls are slower than untraced ones)
    bool trace = false;
    double trace_t = 0;
    void trace_mark(const char* what) {
        if (!trace) return;
        (void)hipStreamSynchronize(stream);
        const double t = mxp::now_seconds();
        if (trace_t > 0 && what) fprintf(stderr, "mxp trace %-28s %9.3f ms\n", what, (t - trace_t) * 1e3);
        trace_t = t;
    }
    // host time since the last trace_mark, without synchronising (where the host is in an upload)
    void trace_host(const char* what) const {
        if (!trace || trace_t <= 0) return;
        fprintf(stderr, "mxp trace   (host) %-21s %9.3f ms\n", what, (mxp::now_seconds() - trace_t) * 1e3);
    }
    // the batch's columns copied beside its strings (MXP_PACK_COLS_BESIDE=1) instead of after them
    // (the default: the string passes then run while the columns copy)
    bool pack_cols_beside = false;
    // mxp_batch_upload_ex(MXP_UPLOAD_NO_WAIT): return before the batch's copies are in
    bool upload_no_wait = false;
    // large device -> pageable caller memory through two pinned bounce buffers: the copy of chunk
    // k + 1 overlaps the host threads' copy of chunk k out of pinned memory (a pageable hipMemcpy
    // stages at a fraction of the pinned rate)
    static constexpr size_t kBounce = 32u << 20;
    // downloads into pinned memory from this size on are shader copies (mxp_d2h_copy_kernel), unless
    // d2h_dma (MXP_D2H_DMA=1: the copy engine's DMA, ~30 GB/s on the box against ~54)
    static constexpr size_t kShaderCopyMin = 64u << 10;
    bool d2h_dma = false;
    bool resolve_tile = true;  // Resolve's default-namespace range walked by resolve_tile (MXP_RESOLVE_TILE)
    int resolve_pairs = 1;  // pair Resolve where the plan allows it (MXP_RESOLVE_PAIRS=0: the bitmap; 2: a
                            // Resolve that cannot take it fails -- tests)
    // the device packer's column copies (pack_device.cpp)
    // [0] the packer's copies, [1] small read-backs, [2] the packer's kernels (apart from the engine
    // stream: an event recorded there -- a freed batch's -- then never waits for a later batch's
    // packer, which waits for its copies)
    static constexpr int kCopyStreams = 3;
    hipStream_t copy_s[kCopyStreams] = {};
    hipStream_t copy_stream(int k) {  // (created on first use; null on failure, last_error set)
        if (!copy_s[k]) {
            hipError_t e = hipStreamCreateWithFlags(&copy_s[k], hipStreamNonBlocking);
            if (e != hipSuccess) {
                copy_s[k] = nullptr;
                hipfail(e, "copy stream");
            }
        }
        return copy_s[k];
    }
    void* bounce[2] = {nullptr, nullptr};
    uint32_t* res_small = nullptr;  // pinned: a compact Resolve's error-record and pair-overflow counts
    // the resolver's per-word tables on the device (res_lo / _hi / _amask / _empty) are those of
    // configuration res_gen and this variety (res_tab_key = res_gen << 6 | variety): kept across calls
    uint64_t res_gen = 0, res_tab_key = ~0ull;
    bool res_any_empty = false;
    hipEvent_t bounce_ev[2] = {nullptr, nullptr};
    int download(void* dst, const void* dsrc, size_t bytes, const char* what);
    // several downloads: those into pinned memory queued together with one synchronisation, the
    // others through download()
    struct Piece {
        void* dst;
        const void* src;
        size_t bytes;
    };
    int download_all(const std::vector<Piece>& pieces, const char* what);
    static bool is_pinned(const void* p);
    static void* host_dev_ptr(const void* p);
    hipError_t queue_d2h(void* dst, void* hd, const void* dsrc, size_t bytes);
    DevBuf d_errlog, d_errcount;
    uint32_t errcap = 1u << 23;  // error records kept per batch (MXP_ERRCAP); mxp_error_count counts all

    // last batch error details: key = request << 32 | rule.  The records are kept as the device
    // wrote them (last_recs) and their texts formatted when a pair is asked for: the index over
    // them is built on the first mxp_pair_error, so an evaluation / Resolve pays only the record
    // download.  Conversion errors print the caller's value, so theirs are formatted eagerly (the
    // caller's batch is gone by the time a text is asked for); texts asked for, and the records of
    // recomputed windows, are memoized in last_errors.
    std::unordered_map<uint64_t, std::pair<uint32_t, std::string>> last_errors;
    std::vector<mxp_err_rec, PinnedAlloc<mxp_err_rec>> last_recs;
    std::vector<int32_t> last_rec_text;          // per record: index into last_rec_texts, or -1; empty
                                                 // (or shorter than last_recs): -1 for the rest
    std::vector<std::string> last_rec_texts;
    std::unordered_map<uint64_t, uint32_t> rec_index;  // key -> record (built on first use)
    bool rec_indexed = false;
    // map texts of the last batch ("map[k:v ...]" per map id, the caller's order), kept when its error
    // records overflowed the log and the device batch holds no map contents: a recomputed window's
    // conversion error prints the map after the caller's batch is gone
    std::vector<std::string> snap_maps;
    // the last evaluation's records left on the device until a text is asked for (ensure_recs):
    // recs_pending records in d_errlog_prev, the buffer the next evaluation does not write
    DevBuf d_errlog_prev;
    uint32_t recs_pending = 0;
    bool lazy_records = true;  // MXP_LAZY_RECORDS=0: download every evaluation's records at once
    int ensure_recs();
    void clear_errors() {
        recs_pending = 0;
        snap_maps.clear();
        last_errors.clear();
        last_recs.clear();
        last_rec_text.clear();
        last_rec_texts.clear();
        rec_index.clear();
        rec_indexed = false;
    }
    // resolve scratch (resolver.cpp), reused across calls
    DevBuf res_dm, res_de, res_info, res_lo, res_hi, res_amask, res_empty, res_status, res_err_rule, res_count,
        res_off, res_sel;
    // compact Resolve (resolver.cpp): request error flags instead of the error bitmap, each request's
    // first applicable erroring rule from the error records (sparse pairs scattered into res_err_in),
    // block sums of the device scan of the counts
    DevBuf res_flags, res_err_in, res_pairs, res_bsum, res_stash;
    std::vector<uint32_t> res_best;       // [n] host scratch: best resolution rank per request (~0 none)
    // the namespace names of the configuration on the device (mxp_ns_kernel): open-addressing table
    // of content hashes, descriptors, bytes
    DevBuf res_ns_tab, res_ns_desc, res_ns_blob;
    uint32_t res_ns_mask = 0;
    uint64_t last_error_count = 0;
    std::unique_ptr<mxp_dbatch> last_db;  // keeps the last batch's interned overlays for decoding

    // ---------------------------------------------------------------- LowerTables
    uint32_t intern_string(const std::string& s) override {
        auto it = gstr_ids.find(s);
        if (it != gstr_ids.end()) return it->second;
        uint32_t id = (uint32_t)gstrs.size();
        gstr_ids.emplace(s, id);
        gstrs.push_back(s);
        return id;
    }
    uint64_t intern_bytes(const std::string& raw) override {
        std::string canon = mxp::ip_canonical((const uint8_t*)raw.data(), raw.size());
        return MXP_BYTES_ID(intern_in(gcanon_ids, gcanon, canon), intern_in(gbytes_ids, gbytes, raw));
    }
    static uint32_t intern_in(std::unordered_map<std::string, uint32_t>& ids, std::vector<std::string>& v,
                              const std::string& s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        uint32_t id = (uint32_t)v.size();
        ids.emplace(s, id);
        v.push_back(s);
        return id;
    }
    uint32_t intern_time(int64_t s, int32_t ns) override {
        TimeKey k{s, ns};
        auto it = gtime_ids.find(k);
        if (it != gtime_ids.end()) return it->second;
        uint32_t id = (uint32_t)gtimes.size();
        gtime_ids.emplace(k, id);
        gtimes.push_back(k);
        return id;
    }
    uint32_t column(const std::string& attr) override {
        auto it = col_ids.find(attr);
        if (it != col_ids.end()) return it->second;
        uint32_t id = (uint32_t)cols.size();
        col_ids.emplace(attr, id);
        cols.push_back(attr);
        return id;
    }
    uint32_t vcolumn(const std::string& attr, const std::string& key) override {
        auto k = std::make_pair(attr, key);
        auto it = vcol_ids.find(k);
        if (it != vcol_ids.end()) return it->second;
        uint32_t id = (uint32_t)vcols.size();
        vcol_ids.emplace(k, id);
        vcols.push_back(k);
        intern_string(key);
        return id;
    }
    int32_t attr_type(const std::string& attr) override {
        auto it = vocab.find(attr);
        return it == vocab.end() ? -1 : it->second;
    }
    int32_t regex_const(const std::string& pattern, std::string* err) override {
        auto it = rx_ids.find(pattern);
        if (it != rx_ids.end()) {
            *err = it->second.second;
            return it->second.first;
        }
        mxp::Dfa d;
        std::string e;
        const int rc = mxp::regex_compile({pattern}, kRegexStates, &d, &e);
        int32_t id = rc == mxp::RX_OK ? (int32_t)rx_set.add(d) : rc == mxp::RX_SYNTAX ? -1 : -2;
        if (id >= 0) rx_dfas.push_back(std::move(d));
        rx_ids.emplace(pattern, std::make_pair(id, e));
        *err = e;
        return id;
    }
    bool regex_const_match(int32_t dfa, const std::string& subject) override {
        return mxp::dfa_match_host(rx_dfas[(size_t)dfa], subject);
    }
    void regex_source(int kind, const std::string& attr, const std::string& key, uint32_t sid) override {
        switch (kind) {
        case mxp::RX_SRC_COLUMN: rx_cols.insert(column(attr)); break;
        case mxp::RX_SRC_VCOLUMN: rx_vcols.insert(vcolumn(attr, key)); break;
        case mxp::RX_SRC_MAPVALS: rx_mapcols.insert(column(attr)); break;
        default: rx_consts.insert(sid); break;
        }
    }

    int fail(int code, const std::string& msg) {
        last_error = msg;
        return code;
    }
    int hipfail(hipError_t e, const char* what) {
        last_error = std::string(what) + ": " + hipGetErrorString(e);
        return MXP_ERR_DEVICE;
    }

    void reset_tables() {
        resolver = ResolverConf();  // a new rule set needs a new resolver configuration
        gstr_ids.clear();
        gstrs.clear();
        gbytes_ids.clear();
        gbytes.clear();
        gcanon_ids.clear();
        gcanon.clear();
        gtime_ids.clear();
        gtimes.clear();
        cols.clear();
        col_ids.clear();
        vcols.clear();
        vcol_ids.clear();
        rules.clear();
        have_rules = false;
        recycle(last_db.release());  // the last batch's ids and error records belong to the old rule set
        clear_errors();
        err_windows.clear();
        errors_complete = true;
        need_ipof = need_tsof = need_strings = need_maps = need_rxof = false;
        rx_ids.clear();
        rx_set = mxp::DfaSetHost();
        rx_dfas.clear();
        rx_cols.clear();
        rx_vcols.clear();
        rx_mapcols.clear();
        rx_consts.clear();
        empty_sid = intern_string("");
    }

    // batched runtime.resolver configuration (resolver.cpp)
    struct ResolverConf {
        bool set = false;
        std::string identity, default_ns;
        std::vector<std::string> ns_names;               // namespaces that have rules
        std::unordered_map<std::string, uint32_t> ns_ids;
        std::vector<uint32_t> ns_lo, ns_hi;              // contiguous rule range per namespace
        std::vector<uint32_t> vmask;                     // per rule: varieties with actions
        std::vector<uint8_t> tcp, empty;                 // per rule: TCP rule; empty match
        uint32_t default_id = 0xFFFFFFFFu;
    } resolver;

    int compile(const char* const* exprs, uint32_t n, int32_t* status);
    // the attribute names the compiled set reads (columns, then the maps of map["key"] columns), plus
    // the resolver's identity attribute and context.protocol once it is configured
    std::vector<std::string> read_attributes() const {
        std::vector<std::string> out;
        std::set<std::string> seen;
        auto add = [&](const std::string& s) {
            if (seen.insert(s).second) out.push_back(s);
        };
        for (auto& c : cols) add(c);
        for (auto& v : vcols) add(v.first);
        if (resolver.set) {
            add(resolver.identity);
            add("context.protocol");
        }
        return out;
    }
    std::vector<std::string> attr_names;  // mxp_ruleset_columns' strings (valid until the next call)
    // A caller's batch is checked before any packer (host or device) or host pass reads it: every
    // column the rule set or the resolver reads, the string offsets and the map CSR -- ids past their
    // tables, offsets running backwards, unknown kinds -- so a malformed batch is MXP_ERR_ARG with the
    // first bad field named, never an out-of-range index into a device table (protoBag.go:255-265
    // answers an undefined index with an error too).
    // parts: kCheckStrings (the string table), kCheckColumns (columns and maps); the pointer and
    // name checks always
    static constexpr int kCheckStrings = 1, kCheckColumns = 2;
    int check_batch(const mxp_bag_batch* b, int parts = kCheckStrings | kCheckColumns);
    void recycle(mxp_dbatch* db);  // a batch no longer used: its blocks to the bin (mxp_batch_free)
    // pack + launch into fresh device bitmaps (dm, de; dv = Eval registers when non-null)
    // d_req_err: compact error output (per-request flags; de is not written)
    // ... of a batch already uploaded (mxp_batch_upload; the Resolve of a batch uploaded ahead)
    int evaluate_uploaded(mxp_dbatch* db, DevBuf& dm, DevBuf& de, DevBuf* dv, uint8_t* d_req_err);
    int evaluate(const mxp_bag_batch* batch, DevBuf& dm, DevBuf& de, DevBuf* dv, std::unique_ptr<mxp_dbatch>& db,
                 uint8_t* d_req_err = nullptr);
    // wait for the evaluation, fetch and format its error records, keep `db` as the last batch
    int collect_errors(const mxp_bag_batch* batch, std::unique_ptr<mxp_dbatch>& db);
    int expand_class_errors(const mxp_bag_batch* batch, mxp_dbatch* db, uint32_t n_class, uint32_t room);
    DevBuf d_vtlog;                  // class records of the value-class kernel
    uint32_t vtlog_cap = 1u << 20;
    struct PackedHost {
        std::vector<uint8_t> kinds;
        std::vector<uint64_t> vals, ipof, tsof;
        std::vector<uint32_t> moff, mk, mv, rxof;
        mxp::DfaSetHost rxb;
    };
    mxp::SvMap gstr_view, gbytes_view, gcanon_view;  // string-view indexes of the interning tables
    size_t views_n[3] = {~(size_t)0, 0, 0};
    void build_views();
    int pack_host(const mxp_bag_batch* b, mxp_dbatch* db, PackedHost& H);
    // mxp_batch_upload: the device packer (pack_device.cpp), or the host one (MXP_HOST_PACK=1, and
    // rule sets reading more than MXP_PACK_MAXCOL columns)
    // The batch is checked (check_batch) before any host pass reads it: by the device packer right
    // after it has queued the batch's H2D copies (from pinned caller memory the check overlaps them;
    // no kernel reads the batch before the check has passed), else first.
    int pack(const mxp_bag_batch* b, mxp_dbatch* db) {
        db->res_raw = false;
        const bool dev = !host_pack && cols.size() + vcols.size() <= MXP_PACK_MAXCOL;
        if (!dev && db->wide) db->wide->materialize();  // (the host packer reads the v1 layout)
        if (!dev)
            if (int rc0 = check_batch(b)) return rc0;
        // the device packer returns once the caller's arrays are copied; its kernels run on, and the
        // rest (finish_pack) waits for the batch's first evaluation
        if (dev) return pack_device(b, db);
        int rc = pack_on_host(b, db);
        if (!rc) rc = pack_heads(db);
        if (!rc) rc = pack_dict(db);
        // the batch is complete when the call returns (evaluations run on the caller's streams)
        hipError_t e;
        if (!rc && (e = hipStreamSynchronize(stream)) != hipSuccess) rc = hipfail(e, "pack sync");
        return rc;
    }
    int pack_dict(mxp_dbatch* db);   // the value-class dictionary of the batch (mxp_vt_classify_kernel)
    int pack_heads(mxp_dbatch* db);  // kargs.heads of the probed columns (MXP_HEADS=0: none)
    bool heads_on = true;
    // columns a prefix or composite guard index probes (plan 0's indexes, a superset of every other
    // plan's): heads are built for these alone; head_slot_of[col] is the row (MXP_VM_DONE: none)
    std::vector<uint32_t> head_cols, head_slot_of;
    DevBuf d_head_cols;
    uint32_t* gate_next_out = nullptr;  // eval_device_hits -> launch: the next evaluation's gate word
    hipStream_t stats_stream = nullptr;  // stream of the last stats_ev record (a wait only across streams)
    int pack_on_host(const mxp_bag_batch* b, mxp_dbatch* db);
    int pack_device(const mxp_bag_batch* b, mxp_dbatch* db);
    int pack_device_body(const mxp_bag_batch* b, mxp_dbatch* db);
    int pack_vt_tables(mxp_dbatch* db);  // the value-class tables of the active slots
    bool host_pack = false;
    const mxp_bag_batch2* narrow_src = nullptr;  // the narrow batch pack_device copies (mxp_batch_upload2)
    // device copies of the interning pools (strings: d_gstr / d_gstr_off) and their hash tables:
    // [0] strings [1] byte strings [2] canonical byte strings [3] timestamps
    int ensure_dev_pools();
    bool dp_built = false;
    size_t dp_sizes[4] = {0, 0, 0, 0};
    DevBuf dp_ht[4], dp_desc[2], dp_blob[2], dp_tsec, dp_tnsec;
    uint32_t dp_mask[4] = {0, 0, 0, 0};
    // the rest of a device-packed batch's upload, at its first evaluation (pack_device.cpp): the
    // value-class sizing from the packer's distinct counts, the class tables, heads, dictionary
    int finish_pack(mxp_dbatch* db);
    bool finish_fail_done = false;  // (test hook of finish_pack, MXP_DEBUG_FLAGS 1 << 29)
    void release_pack_scratch(mxp_dbatch* db);  // the packer's scratch no later call reads, to the bin
    uint32_t vcol_key_id(uint32_t j) const {
        auto it = gstr_ids.find(vcols[j].second);
        return it == gstr_ids.end() ? 0xFFFFFFFEu : it->second;
    }
    int wire_decode(const mxp_wire_batch* w, const char* const* names, uint32_t n_names, mxp_wire** out);  // wire.cpp
    void fill_args(mxp_kargs* A, const mxp_dbatch* db, const Plan& P) const;
    int vt_prepare(mxp_dbatch* db, const Plan& P);
    bool vt_fresh = false;  // the last vt_prepare uploaded a batch's tables (on the engine stream)
    uint32_t last_mask = 0;  // value-class slots of the last launch
    uint8_t* req_err_out = nullptr;  // compact error output of the next launch (kargs.req_err)
    const uint32_t* hits_gate_out = nullptr;  // fused-counter gate of the next launch (kargs.hits_gate)
    DevBuf d_gate;                   // u32[2] by evaluation parity: fused counters on (set by the previous
                                     // evaluation's mxp_hits_kernel block (0, 0), next_gate)
    uint32_t gate_par = 0;
    bool wave_times = false;  // MXP_WAVE_TIMES: index kernel waves record {start, end, XCC}
    DevBuf d_wave_t;
    uint32_t wave_t_n = 0;
    // requests [q_lo, q_hi) of the batch (default: all); q_lo a multiple of 4
    int launch(mxp_dbatch* db, hipStream_t s, uint32_t* d_match, uint32_t* d_err, uint64_t* d_vals, bool log,
               unsigned long long* d_hits = nullptr, uint64_t* d_stats = nullptr, uint32_t q_lo = 0,
               uint32_t q_hi = 0xFFFFFFFFu);
    int launch_body(mxp_dbatch* db, hipStream_t s, uint32_t* d_match, uint32_t* d_err, uint64_t* d_vals, bool log,
                    unsigned long long* d_hits, uint64_t* d_stats, uint32_t q_lo, uint32_t q_hi);
    // fused hit counters: the true pairs the guard-index kernel set (d_stats) decide, on the device,
    // between counting in the next evaluation's kernels and the streaming hits kernel (d_gate)
    DevBuf d_stats;
    hipEvent_t stats_ev = nullptr;  // recorded after each evaluation's gate update
    bool stats_pending = false;     // an evaluation with a gate update has been queued
    // columns of a window of requests [q0, q1) of the last batch, downloaded for error texts
    struct ErrWindow {
        uint32_t q0 = 0, q1 = 0, ncol = 0;
        std::vector<uint8_t> kinds;   // [ncol][q1 - q0]
        std::vector<uint64_t> vals;
    };
    std::string format_error(const mxp_bag_batch* b, const mxp_dbatch* db, const mxp_err_rec& r,
                             const ErrWindow* win = nullptr) const;
    std::string packed_value_text(const mxp_dbatch* db, uint32_t kind, uint64_t v) const;
    // Error records are a cache of the error bits: a pair whose bit is set but whose record is
    // missing (log capacity exceeded, MXP_ERRCAP) is recomputed on demand by re-evaluating its
    // window of requests of the last batch with a fresh log (recompute_errors).
    bool errors_complete = true;
    std::set<uint32_t> err_windows;  // windows of the last batch already recomputed
    static constexpr uint32_t kErrWindow = 64;
    uint32_t win_log_cap = 0;           // != 0 while launch() runs a recomputed window
    DevBuf d_winlog, d_wincount;        // that window's error log
    int recompute_errors(uint32_t request);
    // the text of an error pair of the last batch ("" when it did not fail); -1 on a device failure
    int pair_error_text(uint32_t request, uint32_t rule, std::string* text, uint32_t* code);
    int64_t logged_record(uint64_t key);
    std::string string_of(const mxp_dbatch* db, uint64_t sid) const {
        if (!db) db = last_db.get();
        if (sid < gstrs.size()) return gstrs[sid];
        uint64_t j = sid - gstrs.size();
        std::string out;
        return (db && db->overlay_string(j, &out)) ? out : std::string("?");
    }
};

