// pack_device.cpp -- mxp_batch_upload on the device (pack_args.h): the caller's batch goes up as
// given and is interned, gathered and pre-tabled by pack.hip; the host keeps only the column-name
// resolution, the run-time regexp compilation (host DFA builder) and the value-class sizing.
//
// Ids match the host packer's (engine.cpp pack_host) spaces: rule-set pool ids first, then
// batch-local ids -- G + batch string index of the content's representative for strings, and the
// byte-string / canonical / time pools' sizes + item index for the others.  Texts of batch-local
// ids (error messages, Eval values) are read back from the device on demand (mxp_dbatch accessors).
#include <algorithm>
#include <cstring>
#include <string_view>
#include <unordered_map>

#include "engine_impl.h"
#include "pack_args.h"

extern "C" hipError_t mxp_launch_pack(const mxp_pack_args* a, uint32_t step, uint32_t arg, hipStream_t s);
extern "C" hipError_t mxp_launch_widen(const uint32_t* in, uint64_t* out, uint64_t n, hipStream_t s);

namespace {
constexpr size_t kVtBytes = 8 * MXP_PACK_VTCAND;  // value-class distinct counts + overflow flags (u32 pairs)
constexpr uint32_t kRxDirect = 0x80000000u;          // rx pair keyed by an engine string id

uint32_t table_size(uint64_t items) {
    uint64_t n = 64;
    while (n < 2 * items) n <<= 1;
    return (uint32_t)n;
}

// host-built open-addressing table of a rule-set pool (the packer's probe sequence)
std::vector<unsigned long long> pool_table(size_t n, const std::function<std::string(size_t)>& item) {
    std::vector<unsigned long long> t(table_size(n), 0);
    const uint32_t mask = (uint32_t)t.size() - 1;
    for (size_t i = 0; i < n; i++) {
        const std::string v = item(i);
        const uint64_t h = mxp_item_hash((const uint8_t*)v.data(), (uint32_t)v.size());
        uint32_t s = (uint32_t)h & mask;
        while (t[s]) s = (s + 1) & mask;
        t[s] = ((h >> 32) << 32) | (i + 1);
    }
    return t;
}
}  // namespace

// device copies of the rule set's interning pools + their tables (rebuilt when a compile grew them)
int mxp_engine::ensure_dev_pools() {
    const size_t sizes[4] = {gstrs.size(), gbytes.size(), gcanon.size(), gtimes.size()};
    if (dp_built && std::equal(sizes, sizes + 4, dp_sizes)) return MXP_OK;
    hipError_t e;
    auto put = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.alloc(bytes ? bytes : 16)) != hipSuccess) return hipfail(e, what);
        if (bytes && (e = hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice)) != hipSuccess) return hipfail(e, what);
        return MXP_OK;
    };
    int rc;
    auto t_str = pool_table(gstrs.size(), [&](size_t i) { return gstrs[i]; });
    if ((rc = put(dp_ht[0], t_str.data(), t_str.size() * 8, "pool table"))) return rc;
    dp_mask[0] = (uint32_t)t_str.size() - 1;
    const std::vector<std::string>* pools[2] = {&gbytes, &gcanon};
    for (int k = 0; k < 2; k++) {
        std::vector<uint64_t> desc;
        std::string blob;
        if (!string_pool(*pools[k], &desc, &blob)) return fail(MXP_ERR_ARG, "rule-set byte string longer than 16 MiB");
        if ((rc = put(dp_desc[k], desc.data(), desc.size() * 8, "pool desc"))) return rc;
        if ((rc = put(dp_blob[k], blob.data(), blob.size(), "pool blob"))) return rc;
        auto t = pool_table(pools[k]->size(), [&](size_t i) { return (*pools[k])[i]; });
        if ((rc = put(dp_ht[1 + k], t.data(), t.size() * 8, "pool table"))) return rc;
        dp_mask[1 + k] = (uint32_t)t.size() - 1;
    }
    std::vector<int64_t> ts(gtimes.size());
    std::vector<int32_t> tn(gtimes.size());
    for (size_t i = 0; i < gtimes.size(); i++) {
        ts[i] = gtimes[i].s;
        tn[i] = gtimes[i].ns;
    }
    if ((rc = put(dp_tsec, ts.data(), ts.size() * 8, "pool times"))) return rc;
    if ((rc = put(dp_tnsec, tn.data(), tn.size() * 4, "pool times"))) return rc;
    auto t_time = pool_table(gtimes.size(), [&](size_t i) {
        uint8_t k[12];
        mxp_time_key(gtimes[i].s, gtimes[i].ns, k);
        return std::string((const char*)k, 12);
    });
    if ((rc = put(dp_ht[3], t_time.data(), t_time.size() * 8, "pool table"))) return rc;
    dp_mask[3] = (uint32_t)t_time.size() - 1;
    std::copy(sizes, sizes + 4, dp_sizes);
    dp_built = true;
    return MXP_OK;
}

// Any failure after the first copy was queued waits for the copy streams before returning: the
// caller's arrays may still be read by DMA and the packer's kernels may still use the batch's blocks,
// and a failed upload hands no batch back to wait on.  A failed MXP_UPLOAD_NO_WAIT upload
// has finished reading the caller's arrays when it returns.
int mxp_engine::pack_device(const mxp_bag_batch* b, mxp_dbatch* db) {
    const int rc = pack_device_body(b, db);
    if (rc) {
        for (int k : {0, 2})
            if (copy_s[k]) (void)hipStreamSynchronize(copy_s[k]);
    }
    return rc;
}

int mxp_engine::pack_device_body(const mxp_bag_batch* b, mxp_dbatch* db) {
    const uint32_t n = b->n_requests;
    const uint32_t C = (uint32_t)cols.size(), V = (uint32_t)vcols.size();
    const uint32_t ncol = C + V;
    if (ncol > MXP_PACK_MAXCOL) {  // (wider rule sets: pack() checked the batch)
        if (db->wide) db->wide->materialize();
        return pack_on_host(b, db);
    }
    int rc;
    if ((rc = ensure_dev_pools())) return rc;
    hipStream_t s = copy_stream(2);  // (the packer's kernels: their own stream)
    if (!s) return fail(MXP_ERR_DEVICE, last_error);
    hipError_t e;
    PackScratch& P = db->pk;
    db->n = n;
    db->dev_packed = true;
    const uint32_t NS = b->n_strings, NT = b->n_times, NM = b->n_maps;
    const uint32_t G = (uint32_t)gstrs.size();
    const uint64_t S = (uint64_t)G + NS;
    db->ns = NS;
    db->nt = NT;
    db->G = G;
    db->GB = (uint32_t)gbytes.size();
    db->GC = (uint32_t)gcanon.size();
    db->GT = (uint32_t)gtimes.size();
    std::unordered_map<std::string_view, uint32_t> bcol;
    for (uint32_t c = 0; c < b->n_columns; c++) bcol.emplace(b->column_names[c], c);
    std::vector<int32_t> src(ncol, -1);
    bool any_map = need_maps;
    for (uint32_t c = 0; c < ncol; c++) {
        auto it = bcol.find(c < C ? std::string_view(cols[c]) : std::string_view(vcols[c - C].first));
        if (it != bcol.end()) {
            src[c] = (int32_t)it->second;
            any_map |= c >= C;
        }
    }
    auto grow = [&](DevBuf& d, size_t bytes, const char* what) -> int {
        if (d.n >= bytes && d.p) return MXP_OK;
        if ((e = d.alloc(bytes)) != hipSuccess) return hipfail(e, what);
        return MXP_OK;
    };
    // (engine-stream uploads of host vectors of this call: the run-time pattern pairs)
    auto up_s = [&](DevBuf& d, const void* src_p, size_t bytes, const char* what) -> int {
        if ((rc = grow(d, bytes ? bytes : 16, what))) return rc;
        if (bytes && (e = hipMemcpyAsync(d.p, src_p, bytes, hipMemcpyHostToDevice, s)) != hipSuccess)
            return hipfail(e, what);
        return MXP_OK;
    };
    auto alloc = [&](DevBuf& d, size_t bytes, const char* what) -> int {
        if ((e = d.alloc(bytes ? bytes : 16)) != hipSuccess) return hipfail(e, what);
        return MXP_OK;
    };
    // ---- the batch as given, into the batch's own scratch (db->pk), all on the copy stream: the
    // strings (with times and maps) first, then the columns.  The call returns once they are in (the
    // caller's arrays are free again); the packer's kernels on the engine stream wait for them.
    hipStream_t cs = copy_stream(0);
    if (!cs) return fail(MXP_ERR_DEVICE, last_error);
    for (int k = 0; k < 3; k++)
        if (!db->pk_ev[k] && (e = hipEventCreateWithFlags(&db->pk_ev[k], kOrderEvent)) != hipSuccess) {
            db->pk_ev[k] = nullptr;
            return hipfail(e, "pack event");
        }
    auto up = [&](DevBuf& d, const void* src_p, size_t bytes, const char* what) -> int {
        if ((rc = grow(d, bytes ? bytes : 16, what))) return rc;
        if (bytes && (e = hipMemcpyAsync(d.p, src_p, bytes, hipMemcpyHostToDevice, cs)) != hipSuccess)
            return hipfail(e, what);
        return MXP_OK;
    };
    // a narrow batch (mxp_batch_upload2): its u32 arrays go over the link and are widened here, on the
    // copy stream behind their copies (b is its host view)
    const mxp_bag_batch2* nb = narrow_src;
    auto up_wide = [&](DevBuf& d, DevBuf& d32, const uint64_t* src64, const uint32_t* src32, size_t count,
                       const char* what) -> int {
        if (!nb || !src32) return up(d, src64, count * 8, what);
        if ((rc = up(d32, src32, count * 4, what))) return rc;
        if ((rc = grow(d, count ? count * 8 : 16, what))) return rc;
        if (count && (e = mxp_launch_widen(d32.as<uint32_t>(), d.as<uint64_t>(), count, cs)) != hipSuccess)
            return hipfail(e, what);
        return MXP_OK;
    };
    const uint64_t sbytes = NS ? (nb ? (uint64_t)nb->str_offsets32[NS] : b->str_offsets[NS]) : 0;
    if ((rc = up_wide(P.pk_soff, P.pk_soff32, b->str_offsets, nb ? nb->str_offsets32 : nullptr, NS ? (size_t)NS + 1 : 0,
                      "upload string offsets")))
        return rc;
    // (16 bytes of slack: the intern kernel reads strings 8 bytes at a time)
    if ((rc = grow(P.pk_sbytes, sbytes + 16, "upload string bytes"))) return rc;
    if (sbytes && (e = hipMemcpyAsync(P.pk_sbytes.p, b->str_bytes, sbytes, hipMemcpyHostToDevice, cs)) != hipSuccess)
        return hipfail(e, "upload string bytes");
    if ((rc = up(P.pk_tsec, b->time_sec, (size_t)NT * 8, "upload times"))) return rc;
    if ((rc = up(P.pk_tnsec, b->time_nsec, (size_t)NT * 4, "upload times"))) return rc;
    // (the batch's own copy of its times, read by the evaluation)
    if ((rc = up(db->btsec, b->time_sec, (size_t)NT * 8, "times"))) return rc;
    if ((rc = up(db->btnsec, b->time_nsec, (size_t)NT * 4, "times"))) return rc;
    const uint64_t E = (any_map && NM) ? (nb ? (uint64_t)nb->map_offsets32[NM] : b->map_offsets[NM]) : 0;
    if ((rc = up_wide(P.pk_moff, P.pk_moff32, b->map_offsets, nb ? nb->map_offsets32 : nullptr,
                      any_map && NM ? (size_t)NM + 1 : 0, "upload map offsets")))
        return rc;
    if ((rc = up(P.pk_mkey, b->map_keys, E * 4, "upload map keys"))) return rc;
    if ((rc = up(P.pk_mval, b->map_values, E * 4, "upload map values"))) return rc;
    if ((e = hipEventRecord(db->pk_ev[0], cs)) != hipSuccess) return hipfail(e, "strings event");
    // (MXP_PACK_COLS_BESIDE=1: the string passes also wait for the columns, as if copied beside)
    std::vector<int32_t> slot_of(b->n_columns, -1);  // batch column -> upload slot
    uint32_t nup = 0;
    for (uint32_t c = 0; c < ncol; c++)
        if (src[c] >= 0 && slot_of[src[c]] < 0) slot_of[src[c]] = (int32_t)nup++;
    // the resolver's identity and context.protocol columns as given (mxp_ns_kernel reads them with the
    // raw batch strings): the first batch column of each name, uploaded with the rule columns
    int32_t res_bc[2] = {-1, -1};
    db->res_raw = false;
    if (resolver.set) {
        const std::string_view nm[2] = {resolver.identity, "context.protocol"};
        for (int k = 0; k < 2; k++) {
            auto it = bcol.find(nm[k]);
            if (it == bcol.end()) continue;
            res_bc[k] = (int32_t)it->second;
            if (slot_of[it->second] < 0) slot_of[it->second] = (int32_t)nup++;
        }
    }
    // the columns after the strings on the copy stream: the string passes (interning, the aligned
    // pool) run while they are in flight, and the column passes wait for their event
    trace_host("pack: strings queued");
    for (uint32_t bc = 0; bc < b->n_columns; bc++) {
        if (slot_of[bc] < 0) continue;
        if ((rc = up(P.pk_ck[slot_of[bc]], b->kinds[bc], n, "upload columns"))) return rc;
        const bool narrow = nb && nb->narrow[bc];
        if ((rc = up_wide(P.pk_cv[slot_of[bc]], P.pk_cv32[slot_of[bc]], b->values[bc], narrow ? nb->values32[bc] : nullptr,
                          n, "upload columns")))
            return rc;
    }
    if ((e = hipEventRecord(db->pk_ev[1], cs)) != hipSuccess) return hipfail(e, "columns event");
    if (resolver.set) {
        db->res_id_kind = res_bc[0] >= 0 ? P.pk_ck[slot_of[res_bc[0]]].as<uint8_t>() : nullptr;
        db->res_id_val = res_bc[0] >= 0 ? P.pk_cv[slot_of[res_bc[0]]].as<uint64_t>() : nullptr;
        db->res_pr_kind = res_bc[1] >= 0 ? P.pk_ck[slot_of[res_bc[1]]].as<uint8_t>() : nullptr;
        db->res_pr_val = res_bc[1] >= 0 ? P.pk_cv[slot_of[res_bc[1]]].as<uint64_t>() : nullptr;
        db->res_raw = true;
    }
    // ---- the batch's ids and offsets, checked on the host while the copies run (from pinned caller
    // memory they are DMA; pageable memory is staged by the runtime before hipMemcpyAsync returns)
    trace_host("pack: columns queued");
    // (the string table now; the columns and maps before the column passes, the string passes
    // meanwhile on the device)
    if (int rc0 = check_batch(b, kCheckStrings)) {
        (void)hipStreamSynchronize(cs);  // (the copies still read the caller's arrays)
        return rc0;
    }
    trace_host("pack: strings checked");
    // ---- arguments
    mxp_pack_args A;
    memset(&A, 0, sizeof A);
    A.sbytes = P.pk_sbytes.as<uint8_t>();
    A.soff = P.pk_soff.as<uint64_t>();
    A.tsec = P.pk_tsec.as<int64_t>();
    A.tnsec = P.pk_tnsec.as<int32_t>();
    A.moff = P.pk_moff.as<uint64_t>();
    A.mkey = P.pk_mkey.as<uint32_t>();
    A.mval = P.pk_mval.as<uint32_t>();
    A.ns = NS;
    A.nt = NT;
    A.nm = any_map ? NM : 0;
    A.n = n;
    A.n_entries = E;
    A.gdesc = d_gstr_off.as<uint64_t>();
    A.gblob = d_gstr.as<uint8_t>();
    A.G = G;
    A.S = S;
    A.ncol = ncol;
    A.empty_sid = empty_sid;
    for (uint32_t c = 0; c < ncol; c++) {
        A.vkey[c] = c < C ? 0xFFFFFFFFu : vcol_key_id(c - C);
        if (src[c] >= 0) {
            A.ck[c] = P.pk_ck[slot_of[src[c]]].as<uint8_t>();
            A.cv[c] = P.pk_cv[slot_of[src[c]]].as<uint64_t>();
        }
    }
    // id maps and parsed values (scratch), pre-tables and outputs (the batch's)
    const uint64_t nraw = (uint64_t)NS + S;  // byte-string items: batch strings, then parsed ip() values
    const uint64_t ntime = (uint64_t)NT + S;
    if ((rc = grow(P.pk_sid, (size_t)NS * 4 + 16, "string ids"))) return rc;
    if ((rc = grow(P.pk_braw, nraw * 4 + 16, "byte ids"))) return rc;
    if ((rc = grow(P.pk_bcan, nraw * 4 + 16, "canonical ids"))) return rc;
    if ((rc = grow(P.pk_tid, ntime * 4 + 16, "time ids"))) return rc;
    if ((rc = grow(P.pk_use, (size_t)NS + 16, "uses"))) return rc;
    if ((rc = alloc(db->pip, S * 16, "parsed ips"))) return rc;
    if ((rc = alloc(db->pip_ok, S, "parsed ips"))) return rc;
    if ((rc = alloc(db->pts_sec, S * 8, "parsed times"))) return rc;
    if ((rc = alloc(db->pts_nsec, S * 4, "parsed times"))) return rc;
    if ((rc = alloc(db->pts_ok, S, "parsed times"))) return rc;
    A.sid = P.pk_sid.as<uint32_t>();
    A.braw = P.pk_braw.as<uint32_t>();
    A.bcan = P.pk_bcan.as<uint32_t>();
    A.tid = P.pk_tid.as<uint32_t>();
    A.use = P.pk_use.as<uint8_t>();
    A.pip = db->pip.as<uint8_t>();
    A.pip_ok = db->pip_ok.as<uint8_t>();
    A.pts_sec = db->pts_sec.as<int64_t>();
    A.pts_nsec = db->pts_nsec.as<int32_t>();
    A.pts_ok = db->pts_ok.as<uint8_t>();
    A.max_len_out = nullptr;  // (check_batch bounds every string below 16 MiB)
    if ((e = hipMemsetAsync(P.pk_use.p, 0, (size_t)NS + 16, s)) != hipSuccess) return hipfail(e, "reset uses");
    if ((e = hipMemsetAsync(db->pip_ok.p, 0, S, s)) != hipSuccess) return hipfail(e, "reset parsed");
    if ((e = hipMemsetAsync(db->pts_ok.p, 0, S, s)) != hipSuccess) return hipfail(e, "reset parsed");
    auto launch = [&](uint32_t step, uint32_t arg = 0) -> int {
        if ((e = mxp_launch_pack(&A, step, arg, s)) != hipSuccess) return hipfail(e, "launch pack");
        return MXP_OK;
    };
    // one interning pass: items [i0, i1) of `kind` against pool k's table and the batch table
    auto intern = [&](uint32_t kind, uint64_t i0, uint64_t i1, uint64_t items, DevBuf& tab, uint32_t base,
                      uint32_t* out, bool reset) -> int {
        const uint32_t ts = table_size(items);
        if (reset) {  // (also for an empty first range: the parsed values' pass reuses the table)
            if ((rc = grow(tab, (size_t)ts * 8, "intern table"))) return rc;
            if ((e = hipMemsetAsync(tab.p, 0, (size_t)ts * 8, s)) != hipSuccess) return hipfail(e, "reset table");
        }
        if (i1 <= i0) return MXP_OK;
        mxp_pool_view P;
        memset(&P, 0, sizeof P);
        const int k = kind == MXP_IK_STR ? 0 : kind == MXP_IK_RAW ? 1 : kind == MXP_IK_CANON ? 2 : 3;
        P.ht = dp_ht[k].as<unsigned long long>();
        P.mask = dp_mask[k];
        P.n = (uint32_t)dp_sizes[k];
        if (k == 0) {
            P.desc = d_gstr_off.as<uint64_t>();
            P.blob = d_gstr.as<uint8_t>();
        } else if (k < 3) {
            P.desc = dp_desc[k - 1].as<uint64_t>();
            P.blob = dp_blob[k - 1].as<uint8_t>();
        } else {
            P.tsec = dp_tsec.as<int64_t>();
            P.tnsec = dp_tnsec.as<int32_t>();
        }
        A.pool = P;
        A.btab = tab.as<unsigned long long>();
        A.bmask = ts - 1;
        A.kind = kind;
        A.base = base;
        A.i0 = i0;
        A.i1 = i1;
        A.out = out;
        return launch(1);
    };
    // ---- the string and time passes (the columns are still in flight)
    if ((e = hipStreamWaitEvent(s, db->pk_ev[pack_cols_beside ? 1 : 0], 0)) != hipSuccess) return hipfail(e, "strings wait");
    if ((rc = intern(MXP_IK_STR, 0, NS, NS, P.pk_tab[0], G, P.pk_sid.as<uint32_t>(), true))) return rc;
    if ((rc = intern(MXP_IK_TIME, 0, NT, ntime, P.pk_tab[3], db->GT, P.pk_tid.as<uint32_t>(), true))) return rc;
    // (every batch string goes into the overlay pool: batch-local ids name their representative)
    if ((rc = alloc(db->bstr_off, (size_t)NS * 8, "bstr_off"))) return rc;
    if ((rc = alloc(db->bstr, sbytes + 8ull * NS + 16, "bstr"))) return rc;
    if ((e = hipMemsetAsync(db->bstr.p, 0, sbytes + 8ull * NS + 16, s)) != hipSuccess) return hipfail(e, "reset bstr");
    if ((rc = grow(P.pk_scan, ((size_t)NS + 1) * 8, "scan"))) return rc;
    if ((rc = grow(P.pk_scan_blocks, ((size_t)NS / 1024 + 2) * 8, "scan"))) return rc;
    if ((rc = grow(P.pk_scan_max, ((size_t)NS / 1024 + 2) * 4, "scan"))) return rc;
    A.bdesc = db->bstr_off.as<uint64_t>();
    A.bblob = db->bstr.as<uint8_t>();
    A.scan = P.pk_scan.as<uint64_t>();
    A.scan_blocks = P.pk_scan_blocks.as<uint64_t>();
    A.scan_max = P.pk_scan_max.as<uint32_t>();
    if ((rc = launch(4))) return rc;
    // ---- the column passes, after the columns' check and copies
    if (int rc0 = check_batch(b, kCheckColumns)) {
        (void)hipStreamSynchronize(s);  // (the string passes)
        (void)hipStreamSynchronize(cs);
        return rc0;
    }
    trace_host("pack: columns checked");
    if ((e = hipStreamWaitEvent(s, db->pk_ev[1], 0)) != hipSuccess) return hipfail(e, "columns wait");
    if ((rc = launch(0))) return rc;  // BYTES uses
    if ((rc = intern(MXP_IK_RAW, 0, NS, nraw, P.pk_tab[1], db->GB, P.pk_braw.as<uint32_t>(), true))) return rc;
    if ((rc = intern(MXP_IK_CANON, 0, NS, nraw, P.pk_tab[2], db->GC, P.pk_bcan.as<uint32_t>(), true))) return rc;
    // ---- columns, maps
    if ((rc = alloc(db->kinds, (size_t)ncol * n, "kinds"))) return rc;
    if ((rc = alloc(db->vals, (size_t)ncol * n * 8, "vals"))) return rc;
    A.kinds = db->kinds.as<uint8_t>();
    A.vals = db->vals.as<uint64_t>();
    if ((rc = launch(2))) return rc;
    const bool maps_out = need_maps && NM;
    if ((rc = alloc(db->map_off, maps_out ? ((size_t)NM + 1) * 4 : 0, "map_off"))) return rc;
    if ((rc = alloc(db->map_keys, maps_out ? E * 4 : 0, "map_keys"))) return rc;
    if ((rc = alloc(db->map_vals, maps_out ? E * 4 : 0, "map_vals"))) return rc;
    if (maps_out) {
        A.omoff = db->map_off.as<uint32_t>();
        A.omkey = db->map_keys.as<uint32_t>();
        A.omval = db->map_vals.as<uint32_t>();
        if ((rc = launch(3))) return rc;
    }
    // ---- ip() / timestamp() pre-tables: parse every string id, intern the parsed values
    if ((rc = alloc(db->ipof, need_ipof ? S * 8 : 0, "ipof"))) return rc;
    if ((rc = alloc(db->tsof, need_tsof ? S * 8 : 0, "tsof"))) return rc;
    A.ipof = db->ipof.as<uint64_t>();
    A.tsof = db->tsof.as<uint64_t>();
    if (need_ipof) {
        if ((rc = launch(6, 0))) return rc;
        if ((rc = intern(MXP_IK_RAW, NS, nraw, nraw, P.pk_tab[1], db->GB, P.pk_braw.as<uint32_t>(), false))) return rc;
        if ((rc = intern(MXP_IK_CANON, NS, nraw, nraw, P.pk_tab[2], db->GC, P.pk_bcan.as<uint32_t>(), false))) return rc;
        if ((rc = launch(7, 0))) return rc;
    }
    if (need_tsof) {
        if ((rc = launch(6, 1))) return rc;
        if ((rc = intern(MXP_IK_TIME, NT, ntime, ntime, P.pk_tab[3], db->GT, P.pk_tid.as<uint32_t>(), false))) return rc;
        if ((rc = launch(7, 1))) return rc;
    }
    // ---- value classes: distinct values of the candidate columns (read back with the longest
    // string: the one synchronisation of the upload)
    const uint32_t ncand = (uint32_t)std::min<size_t>(vt_cand_col.size(), MXP_PACK_VTCAND);
    const bool vt_on = !(debug_flags & 131072u) && n && ncand;
    db->vtd_ready = false;
    if (vt_on) {
        const uint32_t tiles = (uint32_t)((n + MXP_VTD_TILE - 1) / MXP_VTD_TILE);
        const size_t lists = (size_t)ncand * tiles * MXP_VTD_TILE, tabs = (size_t)ncand * MXP_VTD_CAP;
        if ((rc = grow(P.pk_vtd_lkey, lists * 8, "vt lists"))) return rc;
        if ((rc = grow(P.pk_vtd_lcr, lists * 8, "vt lists"))) return rc;
        if ((rc = grow(P.pk_vtd_ln, (size_t)ncand * tiles * 4, "vt lists"))) return rc;
        if ((rc = grow(P.pk_vtd_tkey, tabs * 8, "vt tables"))) return rc;
        if ((rc = grow(P.pk_vtd_tcr, tabs * 8, "vt tables"))) return rc;
        if ((rc = grow(P.pk_vtd_meta, kVtBytes, "vt counts"))) return rc;
        if ((e = hipMemsetAsync(P.pk_vtd_tkey.p, 0xFF, tabs * 8, s)) != hipSuccess) return hipfail(e, "reset vt");
        if ((e = hipMemsetAsync(P.pk_vtd_tcr.p, 0, tabs * 8, s)) != hipSuccess) return hipfail(e, "reset vt");
        if ((e = hipMemsetAsync(P.pk_vtd_meta.p, 0, kVtBytes, s)) != hipSuccess) return hipfail(e, "reset vt");
        A.vtd_lkey = P.pk_vtd_lkey.as<unsigned long long>();
        A.vtd_lcr = P.pk_vtd_lcr.as<uint2>();
        A.vtd_ln = P.pk_vtd_ln.as<uint32_t>();
        A.vtd_tkey = P.pk_vtd_tkey.as<unsigned long long>();
        A.vtd_tcr = P.pk_vtd_tcr.as<uint2>();
        A.vtd_meta = P.pk_vtd_meta.as<uint32_t>();
        A.vtd_tiles = tiles;
        for (uint32_t a = 0; a < ncand; a++) A.vt_col[a] = vt_cand_col[a];
        A.n_vt_cand = ncand;
        if ((rc = launch(5))) return rc;
    }
    // run-time regexp patterns meanwhile: the distinct batch strings of the pattern columns
    std::vector<uint32_t> rx_s, rx_v;
    mxp::DfaSetHost rxb;
    if (need_rxof) {
        if (db->wide) db->wide->materialize();  // (a narrow upload: this pass reads the v1 layout)
        std::vector<uint8_t> seen(NS, 0);
        std::unordered_map<std::string_view, uint32_t> by_text;
        auto text_of = [&](uint64_t sidx) {
            return std::string_view((const char*)b->str_bytes + b->str_offsets[sidx],
                                    (size_t)(b->str_offsets[sidx + 1] - b->str_offsets[sidx]));
        };
        auto add = [&](std::string_view t, uint32_t key) {  // key: batch string, or kRxDirect | engine id
            auto it = by_text.find(t);
            uint32_t val;
            if (it != by_text.end()) {
                val = it->second;
            } else {
                mxp::Dfa d;
                std::string err;
                const int rrc = mxp::regex_compile({std::string(t)}, kRegexStates, &d, &err);
                val = rrc == mxp::RX_OK ? rxb.add(d) : rrc == mxp::RX_SYNTAX ? MXP_RXOF_SYNTAX : MXP_RXOF_UNSUPPORTED;
                by_text.emplace(t, val);
            }
            rx_s.push_back(key);
            rx_v.push_back(val);
        };
        bool empty_done = false;
        for (uint32_t c : rx_pattern_cols()) {
            if (c >= ncol || src[c] < 0) continue;
            const uint8_t* k = b->kinds[src[c]];
            const uint64_t* v = b->values[src[c]];
            for (uint32_t q = 0; q < n; q++) {
                uint64_t sv = v[q];
                if (c >= C) {  // a virtual map[key] column: the entry's value, or "" without one
                    if (k[q] != MXP_STRING_MAP) continue;
                    sv = ~0ull;
                    const std::string_view key(vcols[c - C].second);
                    for (uint64_t e2 = b->map_offsets[v[q]]; e2 < b->map_offsets[v[q] + 1]; e2++)
                        if (text_of(b->map_keys[e2]) == key) {
                            sv = b->map_values[e2];
                            break;
                        }
                    if (sv == ~0ull) {
                        if (!empty_done) add(std::string_view(), kRxDirect | empty_sid);
                        empty_done = true;
                        continue;
                    }
                } else if (k[q] != MXP_STRING) {
                    continue;
                }
                if (sv >= NS || seen[sv]) continue;
                seen[sv] = 1;
                add(text_of(sv), (uint32_t)sv);
            }
        }
        // every value of a map whose lookups with run-time keys are patterns
        for (uint32_t c : rx_mapcols) {
            if (c >= ncol || src[c] < 0) continue;
            const uint8_t* k = b->kinds[src[c]];
            const uint64_t* v = b->values[src[c]];
            for (uint32_t q = 0; q < n; q++) {
                if (k[q] != MXP_STRING_MAP) continue;
                for (uint64_t e2 = b->map_offsets[v[q]]; e2 < b->map_offsets[v[q] + 1]; e2++) {
                    const uint64_t sv = b->map_values[e2];
                    if (sv >= NS || seen[sv]) continue;
                    seen[sv] = 1;
                    add(text_of(sv), (uint32_t)sv);
                }
            }
        }
        // rule-set constants that reach a pattern (`m["k"] | "^x"`), by their engine string id
        for (uint32_t sid_c : rx_consts) add(std::string_view(gstrs[sid_c]), kRxDirect | sid_c);
    }
    if ((rc = alloc(db->rxof, need_rxof ? S * 4 : 0, "rxof"))) return rc;
    if (need_rxof) {
        if ((rc = up_s(P.pk_rx, rx_s.data(), rx_s.size() * 4, "upload patterns"))) return rc;
        if ((rc = up_s(P.pk_rxv, rx_v.data(), rx_v.size() * 4, "upload patterns"))) return rc;
        A.rx_s = P.pk_rx.as<uint32_t>();
        A.rx_v = P.pk_rxv.as<uint32_t>();
        A.n_rx = (uint32_t)rx_s.size();
        A.rxof = db->rxof.as<uint32_t>();
        if ((rc = launch(8))) return rc;
    }
    db->rx_nfa = rxb.has_nfa();
    db->rx_wmax = rxb.nfa_wmax();
    auto upd = [&](DevBuf& d, const void* src_p, size_t bytes, const char* what) -> int {
        if ((rc = alloc(d, bytes, what))) return rc;
        if (bytes && (e = hipMemcpyAsync(d.p, src_p, bytes, hipMemcpyHostToDevice, s)) != hipSuccess)
            return hipfail(e, what);
        return MXP_OK;
    };
    if ((rc = upd(db->rx_hdr, rxb.hdr.data(), rxb.hdr.size() * sizeof(mxp_dfa_hdr), "upload rx hdr"))) return rc;
    if ((rc = upd(db->rx_trans, rxb.trans.data(), rxb.trans.size() * 4, "upload rx trans"))) return rc;
    if ((rc = upd(db->rx_ascii, rxb.ascii.data(), rxb.ascii.size() * 2, "upload rx ascii"))) return rc;
    if ((rc = upd(db->rx_hilo, rxb.hilo.data(), rxb.hilo.size() * 4, "upload rx hilo"))) return rc;
    if ((rc = upd(db->rx_hicls, rxb.hicls.data(), rxb.hicls.size() * 2, "upload rx hicls"))) return rc;
    trace_host("pack: all queued");
    // the packer's kernels run on; the call returns once the caller's arrays are copied (the
    // pattern tables above came from host vectors of this call: synchronous then, a rare path)
    if ((e = hipEventRecord(db->pk_ev[2], s)) != hipSuccess) return hipfail(e, "pack event");
    if (need_rxof || !rxb.hdr.empty()) {
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return hipfail(e, "pack sync");
    }
    if (!upload_no_wait && (e = hipEventSynchronize(db->pk_ev[1])) != hipSuccess) return hipfail(e, "pack copies");
    trace_host("pack: copies done");
    db->pack_pending = true;
    db->pk_vt_on = vt_on;
    db->pk_ncand = ncand;
    db->vt_mask = 0;
    return MXP_OK;
}

// The rest of a device-packed batch's upload, before its first evaluation: the value-class sizing
// (pack_host's rule: the first MXP_VT_MAX candidates with few classes) from the packer's distinct
// counts, the class tables, the string heads and the dictionary.  Waits for the packer's kernels.
int mxp_engine::finish_pack(mxp_dbatch* db) {
    if (!db->pack_pending) return MXP_OK;
    hipError_t e;
    if ((e = hipEventSynchronize(db->pk_ev[2])) != hipSuccess) return hipfail(e, "pack sync");
    // (pack_pending stays set until every step below has succeeded: a failed finish -- an allocation
    // of the class tables, say -- leaves the batch unfinished, so a later evaluation of it runs the
    // whole finish again instead of launching with half-built tables)
    // (read back on a stream of its own: the engine stream may already hold a later batch's packer,
    // waiting for that batch's copies)
    uint32_t meta[2 * MXP_PACK_VTCAND] = {};  // distinct keys, overflow
    if (db->pk_vt_on) {
        hipStream_t rb = copy_stream(1);
        if (!rb) return fail(MXP_ERR_DEVICE, last_error);
        if ((e = hipMemcpyAsync(meta, db->pk.pk_vtd_meta.p, kVtBytes, hipMemcpyDeviceToHost, rb)) != hipSuccess ||
            (e = hipStreamSynchronize(rb)) != hipSuccess)
            return hipfail(e, "read back");
    }
    const uint32_t n = db->n;
    db->vt_mask = 0;
    db->vt_capc.assign(vt_cand_col.size(), 0);
    if (db->pk_vt_on) {
        uint32_t active = 0;
        const bool force = (debug_flags & 262144u) != 0;
        db->vtd_ready = true;
        for (uint32_t a = 0; a < db->pk_ncand && active < MXP_VT_MAX; a++) {
            const uint64_t D = meta[2 * a];
            if (meta[2 * a + 1] || D > kVtMaxClasses || (!force && D * 16 > n)) continue;
            uint32_t cap = 64;
            while (cap < 2 * D) cap <<= 1;
            db->vt_capc[a] = cap;
            db->vt_mask |= 1u << a;
            active++;
        }
    }
    // (the batch's tables drawn from the bin, as at upload)
    BlockBin* take0 = g_bin_take;
    const void* db0 = g_bin_db;
    const size_t sz0 = g_bin_db_size;
    g_bin_take = &bin;
    g_bin_db = db;
    g_bin_db_size = sizeof(mxp_dbatch);
    int rc = pack_vt_tables(db);
    // (MXP_DEBUG_FLAGS 1 << 29, tests only: the next finish fails here once, after the class tables)
    if (!rc && (debug_flags & (1u << 29)) && !finish_fail_done) {
        finish_fail_done = true;
        rc = fail(MXP_ERR_NOMEM, "injected finish_pack failure");
    }
    if (!rc) rc = pack_heads(db);
    if (!rc) rc = pack_dict(db);
    g_bin_take = take0;
    g_bin_db = db0;
    g_bin_db_size = sz0;
    if (rc) return rc;
    // (pk_ev[3]: the batch ready on the engine stream -- tables, heads and dictionary too)
    if (!db->pk_ev[3] && (e = hipEventCreateWithFlags(&db->pk_ev[3], kOrderEvent)) != hipSuccess) {
        db->pk_ev[3] = nullptr;
        return hipfail(e, "pack event");
    }
    if ((e = hipEventRecord(db->pk_ev[3], stream)) != hipSuccess) return hipfail(e, "pack event");
    db->pack_pending = false;
    release_pack_scratch(db);
    return MXP_OK;
}

// The packer's scratch that no later call reads goes to the bin once finish_pack's kernels are done
// (an event on the engine stream; the packer stream's kernels finished before finish_pack began):
// everything in db->pk but the batch's string table and the resolver's raw identity / protocol
// columns (the Resolve's device namespaces, mxp_ns_kernel).  A batch kept for double buffering then
// holds its packed image, not the packer's inputs and tables.
void mxp_engine::release_pack_scratch(mxp_dbatch* db) {
    BlockBin::Group g;
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, kOrderEvent) != hipSuccess || hipEventRecord(ev, stream) != hipSuccess) {
        if (ev) (void)hipEventDestroy(ev);
        (void)hipGetLastError();
        return;  // (keep the scratch: freed with the batch)
    }
    g.evs.push_back(ev);
    PackScratch& P = db->pk;
    const void* keep[4] = {db->res_id_kind, db->res_id_val, db->res_pr_kind, db->res_pr_val};
    auto give = [&](DevBuf& d) {
        for (const void* k : keep)
            if (k && k == d.p) return;
        d.reset();
    };
    g_bin_give = &g.blks;
    for (DevBuf* d : {&P.pk_tsec, &P.pk_tnsec, &P.pk_moff, &P.pk_mkey, &P.pk_mval, &P.pk_sid, &P.pk_braw, &P.pk_bcan,
                      &P.pk_tid, &P.pk_use, &P.pk_scan, &P.pk_scan_blocks, &P.pk_scan_max, &P.pk_vtd_lkey, &P.pk_vtd_lcr,
                      &P.pk_vtd_ln, &P.pk_vtd_tkey, &P.pk_vtd_tcr, &P.pk_vtd_meta, &P.pk_rx, &P.pk_rxv, &P.pk_soff32,
                      &P.pk_moff32})
        give(*d);
    for (auto& d : P.pk_tab) give(d);
    for (auto& d : P.pk_ck) give(d);
    for (auto& d : P.pk_cv) give(d);
    for (auto& d : P.pk_cv32) give(d);
    g_bin_give = nullptr;
    if (g.blks.empty()) {
        (void)hipEventDestroy(ev);
        return;
    }
    bin.put(std::move(g));
}
