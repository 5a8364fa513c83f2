// wire.cpp -- CompressedAttributes messages -> columnar batch (mxp_wire_decode, include/mxp.h).
//
// Restates how ProtoBag.Get reads a CheckRequest's attributes (mixer/pkg/attribute/protoBag.go):
//   NewProtoBag :49-65   message dictionary: word i -> index -i-1 (slotToIndex), later words win
//   getIndex    :242-252 a name's index: the message dictionary first, then the global dictionary
//   lookup      :255-266 index >= 0 -> global word, < 0 -> message word -index-1, else an error
//   internalGet :161-239 probe order Strings (value looked up; error -> not found), StringMaps
//                        (every key and value looked up; error -> not found), Int64S, Doubles,
//                        Bools, Timestamps, Durations, Bytes
// The batch's string table is the global words, then every request's message words, then the Bytes
// values, so string values need no copy: a dictionary index maps straight to a batch string id.
#include <cstring>
#include <string_view>

#include "engine_impl.h"

struct mxp_wire {
    std::vector<std::string> names;
    std::vector<const char*> name_ptrs;
    std::vector<std::vector<uint8_t>> kinds;
    std::vector<std::vector<uint64_t>> vals;
    std::vector<const uint8_t*> kind_ptrs;
    std::vector<const uint64_t*> val_ptrs;
    std::string str_bytes;
    std::vector<uint64_t> str_offsets;
    std::vector<int64_t> tsec;
    std::vector<int32_t> tnsec;
    std::vector<uint64_t> map_offsets;
    std::vector<uint32_t> map_keys, map_values;
    mxp_bag_batch view;
};

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// first entry of request q's CSR field whose key is idx (Go map keys are unique)
inline uint64_t find_key(const uint64_t* off, const int32_t* key, uint64_t q, int64_t idx) {
    if (!off) return ~0ull;
    for (uint64_t e = off[q]; e < off[q + 1]; e++)
        if (key[e] == idx) return e;
    return ~0ull;
}

}  // namespace

int mxp_engine::wire_decode(const mxp_wire_batch* w, const char* const* names, uint32_t n_names, mxp_wire** out) {
    if (!w || !out || (n_names && !names)) return MXP_ERR_ARG;
    if (!w->global_offsets || !w->words_off || !w->word_offsets) return fail(MXP_ERR_ARG, "wire batch: missing dictionaries");
    auto* W = new (std::nothrow) mxp_wire();
    if (!W) return MXP_ERR_NOMEM;
    std::unique_ptr<mxp_wire> own(W);
    // columns
    if (names) {
        for (uint32_t i = 0; i < n_names; i++) W->names.emplace_back(names[i] ? names[i] : "");
    } else {
        if (!have_rules) return fail(MXP_ERR_STATE, "no rule set compiled (names = NULL decodes its attributes)");
        W->names = read_attributes();
    }
    const uint32_t C = (uint32_t)W->names.size();
    const uint32_t n = w->n_requests;
    const uint32_t G = w->n_global;
    const uint64_t NW = w->words_off[n];
    const uint64_t NB = w->byt_off ? w->byt_off[n] : 0;
    const uint64_t NT = w->ts_off ? w->ts_off[n] : 0;
    if ((uint64_t)G + NW + NB >= kNone) return fail(MXP_ERR_ARG, "wire batch: too many strings");
    // string table: global words, message words, bytes values
    {
        const uint64_t g0 = w->global_offsets[0], g1 = w->global_offsets[G];
        const uint64_t w0 = w->word_offsets[0], w1 = w->word_offsets[NW];
        const uint64_t b0 = NB ? w->byt_val_off[0] : 0, b1 = NB ? w->byt_val_off[NB] : 0;
        W->str_bytes.reserve((g1 - g0) + (w1 - w0) + (b1 - b0) + 1);
        W->str_bytes.append((const char*)w->global_bytes + g0, g1 - g0);
        W->str_bytes.append((const char*)w->word_bytes + w0, w1 - w0);
        if (NB) W->str_bytes.append((const char*)w->byt_bytes + b0, b1 - b0);
        W->str_bytes.push_back('\0');
        W->str_offsets.resize((size_t)G + NW + NB + 1);
        for (uint32_t i = 0; i <= G; i++) W->str_offsets[i] = w->global_offsets[i] - g0;
        const uint64_t sw = g1 - g0;
        for (uint64_t i = 0; i <= NW; i++) W->str_offsets[G + i] = sw + w->word_offsets[i] - w0;
        const uint64_t sb = sw + (w1 - w0);
        for (uint64_t i = 0; i <= NB; i++) W->str_offsets[G + NW + i] = sb + (NB ? w->byt_val_off[i] - b0 : 0);
    }
    if (NT) {
        W->tsec.assign(w->ts_sec, w->ts_sec + NT);
        W->tnsec.assign(w->ts_nsec, w->ts_nsec + NT);
    }
    // name -> column; each column's global index (globalDict: later duplicates win)
    std::unordered_map<std::string_view, uint32_t, mxp::SvHash> col_of;
    for (uint32_t c = 0; c < C; c++) col_of.emplace(std::string_view(W->names[c]), c);
    std::vector<int64_t> gidx(C, INT64_MIN);
    for (uint32_t i = 0; i < G; i++) {
        const std::string_view v((const char*)w->global_bytes + w->global_offsets[i],
                                 (size_t)(w->global_offsets[i + 1] - w->global_offsets[i]));
        auto it = col_of.find(v);
        if (it != col_of.end()) gidx[it->second] = i;
    }
    // lookup(): a dictionary index of request q -> batch string id (kNone: undefined)
    auto sid_of = [&](uint64_t q, int64_t idx) -> uint32_t {
        if (idx >= 0) return idx < (int64_t)G ? (uint32_t)idx : kNone;
        const uint64_t slot = (uint64_t)(-(idx + 1));
        return slot < w->words_off[q + 1] - w->words_off[q] ? (uint32_t)(G + w->words_off[q] + slot) : kNone;
    };
    // convertStringMap (protoBag.go:269-286): the entries of wire map e as batch string ids.  Two
    // indices naming the same word collide in the Go map and which value survives follows Go's
    // random map order; the batch keeps the first entry in wire order (keys stay unique,
    // mxp_batch.h).  Returns the pair count; writes them when keys / vals are given.
    auto str_at = [&](uint32_t s) {
        return std::string_view(W->str_bytes.data() + W->str_offsets[s], (size_t)(W->str_offsets[s + 1] - W->str_offsets[s]));
    };
    auto map_pairs = [&](uint64_t q, uint64_t e, uint32_t* keys, uint32_t* vals) -> uint64_t {
        uint64_t cnt = 0;
        for (uint64_t x = w->sm_ent_off[e]; x < w->sm_ent_off[e + 1]; x++) {
            const uint32_t ks = sid_of(q, w->sm_ent_key[x]);
            bool dup = false;
            for (uint64_t y = w->sm_ent_off[e]; y < x && !dup; y++) dup = str_at(sid_of(q, w->sm_ent_key[y])) == str_at(ks);
            if (dup) continue;
            if (keys) {
                keys[cnt] = ks;
                vals[cnt] = sid_of(q, w->sm_ent_val[x]);
            }
            cnt++;
        }
        return cnt;
    };
    W->kinds.assign(C, std::vector<uint8_t>(n, MXP_ABSENT));
    W->vals.assign(C, std::vector<uint64_t>(n, 0));
    std::vector<uint32_t> nmaps(n, 0);
    std::vector<uint64_t> npairs(n, 0);
    mxp::par_for(n, 2048, [&](uint64_t q0, uint64_t q1, unsigned) {
        std::vector<int64_t> idx(C);
        for (uint64_t q = q0; q < q1; q++) {
            for (uint32_t c = 0; c < C; c++) idx[c] = gidx[c];
            for (uint64_t s = w->words_off[q]; s < w->words_off[q + 1]; s++) {
                const std::string_view v((const char*)w->word_bytes + w->word_offsets[s],
                                         (size_t)(w->word_offsets[s + 1] - w->word_offsets[s]));
                auto it = col_of.find(v);
                if (it != col_of.end()) idx[it->second] = -(int64_t)(s - w->words_off[q]) - 1;
            }
            for (uint32_t c = 0; c < C; c++) {
                if (idx[c] == INT64_MIN) continue;  // in neither dictionary
                const int64_t x = idx[c];
                uint8_t& k = W->kinds[c][q];
                uint64_t& v = W->vals[c][q];
                uint64_t e;
                if ((e = find_key(w->str_off, w->str_key, q, x)) != ~0ull) {
                    const uint32_t s = sid_of(q, w->str_val[e]);
                    if (s != kNone) k = MXP_STRING, v = s;
                } else if ((e = find_key(w->sm_off, w->sm_key, q, x)) != ~0ull) {
                    bool ok = true;
                    for (uint64_t p = w->sm_ent_off[e]; ok && p < w->sm_ent_off[e + 1]; p++)
                        ok = sid_of(q, w->sm_ent_key[p]) != kNone && sid_of(q, w->sm_ent_val[p]) != kNone;
                    if (ok) {
                        k = MXP_STRING_MAP;
                        v = e;  // the wire entry; renumbered below
                        nmaps[q]++;
                        npairs[q] += map_pairs(q, e, nullptr, nullptr);
                    }
                } else if ((e = find_key(w->i64_off, w->i64_key, q, x)) != ~0ull) {
                    k = MXP_INT64, v = (uint64_t)w->i64_val[e];
                } else if ((e = find_key(w->dbl_off, w->dbl_key, q, x)) != ~0ull) {
                    k = MXP_DOUBLE;
                    memcpy(&v, &w->dbl_val[e], 8);
                } else if ((e = find_key(w->bool_off, w->bool_key, q, x)) != ~0ull) {
                    k = MXP_BOOL, v = w->bool_val[e] ? 1u : 0u;
                } else if ((e = find_key(w->ts_off, w->ts_key, q, x)) != ~0ull) {
                    k = MXP_TIMESTAMP, v = e;
                } else if ((e = find_key(w->dur_off, w->dur_key, q, x)) != ~0ull) {
                    k = MXP_DURATION, v = (uint64_t)w->dur_val[e];
                } else if ((e = find_key(w->byt_off, w->byt_key, q, x)) != ~0ull) {
                    k = MXP_BYTES, v = G + NW + e;
                }
            }
        }
    });
    // string maps: ids and pairs in request order
    std::vector<uint64_t> map_base(n + 1, 0), pair_base(n + 1, 0);
    for (uint32_t q = 0; q < n; q++) {
        map_base[q + 1] = map_base[q] + nmaps[q];
        pair_base[q + 1] = pair_base[q] + npairs[q];
    }
    if (map_base[n] >= kNone || pair_base[n] >= kNone) return fail(MXP_ERR_ARG, "wire batch: too many map entries");
    W->map_offsets.assign(map_base[n] + 1, 0);
    W->map_keys.resize(pair_base[n]);
    W->map_values.resize(pair_base[n]);
    mxp::par_for(n, 2048, [&](uint64_t q0, uint64_t q1, unsigned) {
        for (uint64_t q = q0; q < q1; q++) {
            uint64_t m = map_base[q], p = pair_base[q];
            for (uint32_t c = 0; c < C; c++) {
                if (W->kinds[c][q] != MXP_STRING_MAP) continue;
                const uint64_t e = W->vals[c][q];
                W->vals[c][q] = m;
                p += map_pairs(q, e, W->map_keys.data() + p, W->map_values.data() + p);
                W->map_offsets[m + 1] = p;
                m++;
            }
        }
    });
    for (auto& s : W->names) W->name_ptrs.push_back(s.c_str());
    for (uint32_t c = 0; c < C; c++) {
        W->kind_ptrs.push_back(W->kinds[c].data());
        W->val_ptrs.push_back(W->vals[c].data());
    }
    mxp_bag_batch& B = W->view;
    memset(&B, 0, sizeof B);
    B.n_requests = n;
    B.n_columns = C;
    B.column_names = W->name_ptrs.data();
    B.kinds = W->kind_ptrs.data();
    B.values = W->val_ptrs.data();
    B.n_strings = (uint32_t)(W->str_offsets.size() - 1);
    B.str_bytes = (const uint8_t*)W->str_bytes.data();
    B.str_offsets = W->str_offsets.data();
    B.n_times = (uint32_t)NT;
    B.time_sec = W->tsec.data();
    B.time_nsec = W->tnsec.data();
    B.n_maps = (uint32_t)map_base[n];
    B.map_offsets = W->map_offsets.data();
    B.map_keys = W->map_keys.data();
    B.map_values = W->map_values.data();
    *out = own.release();
    return MXP_OK;
}

extern "C" {

int mxp_wire_decode(mxp_engine* eng, const mxp_wire_batch* wire, const char* const* names, uint32_t n_names,
                    mxp_wire** out) {
    if (!eng) return MXP_ERR_ARG;
    return eng->wire_decode(wire, names, n_names, out);
}

const mxp_bag_batch* mxp_wire_view(const mxp_wire* w) { return w ? &w->view : nullptr; }

void mxp_wire_free(mxp_wire* w) { delete w; }

}  // extern "C"
