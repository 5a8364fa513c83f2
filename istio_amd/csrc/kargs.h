// kargs.h -- argument block of the evaluation kernel (passed by value, lives in the kernarg segment).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

#include "dfa_dev.h"
#include "vm.h"

#define MXP_RXOF_SYNTAX 0xFFFFFFFFu
#define MXP_RXOF_UNSUPPORTED 0xFFFFFFFEu

// quads per fill-chunk row of the deferred-pair slots (kargs.dtp_slots, 16 B a quad) and counts
// (kargs.dtp_qn, 1 B): the tiles' 256 quads each plus 8 -- a row of exactly 2^k quads (4 MB of slots
// at 1M requests) would put every chunk's same quads on aliased HBM channels
#define MXP_DTP_ROW(tiles) ((uint64_t)(tiles) * 256u + 8u)

// requests per row of the value-class indexes (kargs.vt_cls, u16): the batch's n rounded up to 4
// plus 64 -- rows exactly 2^k requests apart would alias HBM channels across the fill's slots
#define MXP_VT_PITCH(n) ((((uint64_t)(n) + 3u) & ~(uint64_t)3u) + 64u)

typedef struct mxp_kargs {
    // rule set (uploaded once per config snapshot)
    const mxp_vm_ins* prog;      // all rules' programs, concatenated
    const uint32_t* rule_off;    // [n_rules + 1]
    const mxp_guard* guards;     // [n_rules] leading-atom guards (vmopt.h)
    const mxp_rgroup* groups;     // [n_words] per-group guard masks
    const uint32_t* glist;       // groups this launch evaluates (ids into groups)
    const mxp_fill* fills;       // mxp_fill_kernel: chunks of uniform indexed groups
    uint32_t n_glist;
    uint32_t pad3;
    const mxp_seg* segs;         // column segments of the groups
    const uint64_t* gk;          // [n_words * 32] guard constants (0 for unguarded slots)
    const mxp_tmpl* tmpls;       // continuation templates
    const uint32_t* rule_tmpl;   // [n_rules] template of the rule's continuation (~0: none)
    const uint32_t* rule_tmpl2;  // [n_rules] composite-indexed rules: template resuming after the second atom
    const uint32_t* alias_off;   // [n_rules + 1] CSR of duplicate indexed rules (nullptr: none)
    const uint32_t* aliases;
    const uint8_t* dense_of;     // [n_rules] dense canonical id (< 64) of indexed rules with many aliases, 0xFF none (nullptr: none)
    const uint32_t* inj;         // [n_inj][MXP_INJ_SLOT] injection slots of the words holding dense rules
    uint64_t* dense_cm;          // [n] per request: the dense rules found true (index kernel -> inject kernel)
    uint32_t n_inj;
    uint32_t pad5;
    const uint64_t* rconst;      // [n_rules][MXP_VM_MAXREG] per-rule template constants
    const mxp_index* idx;        // guard indexes (mxp_index_kernel)
    const mxp_hent* hents;
    const uint32_t* hbits;       // occupancy bitmaps of the prefix / composite pair tables (mxp_index.boff);
                                 // null: probes load the entry pair first (MXP_DEBUG_FLAGS 4)
    const uint32_t* postings;    // rules of each index entry; with post_tmpl: rule | code << 23 (code = the
                                 // continuation template, 511 direct, 510 look up rule_tmpl / rule_tmpl2)
    const uint32_t* plens;       // prefix indexes: distinct key lengths
    uint32_t n_idx;
    uint32_t lean_cols;          // mxp_guard2_kernel: columns < MXP_CC its groups read (preloaded)
    uint32_t n_rules;
    uint32_t n_words;            // ceil(n_rules / 32)
    uint32_t groups_per_wave;
    uint32_t n;                  // requests in the batch (row stride of columns and bitmaps)
    uint32_t q0, q1;             // requests [q0, q1) this launch evaluates (pipelined chunks)
    uint32_t fill_span;          // mxp_fill_kernel: 256-request spans per wave (MXP_FILL_SPAN)
    // columns: [n_cols][n] kinds / values (resolve columns, then virtual map[key] columns)
    const uint8_t* kinds;
    const uint64_t* vals;
    // interned strings: ids < n_gstr live in the rule set's pool, the rest in the batch pool
    uint64_t n_gstr;
    const uint64_t* gstr_off;    // [n_gstr] offset << 24 | length (8-aligned pool, engine.cpp string_pool)
    const uint8_t* gstr;
    const uint64_t* bstr_off;    // batch overlay strings, same encoding
    const uint8_t* bstr;
    uint32_t empty_sid;
    uint32_t pad0;
    // per-request string maps (CSR over batch map ids)
    const uint32_t* map_off;
    const uint32_t* map_keys;
    const uint32_t* map_vals;
    // per-string pre-tables (ip(), timestamp()); ~0 = conversion error
    const uint64_t* ipof;
    const uint64_t* tsof;
    // regexp DFAs: constant patterns of the rule set; run-time patterns of the batch, reached through
    // rxof[pattern string id] (DFA index in rx_batch, or MXP_RXOF_SYNTAX / MXP_RXOF_UNSUPPORTED)
    mxp_dfa_set rx;
    mxp_dfa_set rx_batch;
    const uint32_t* rxof;
    // outputs
    uint32_t* out_match;         // [n_words][n]
    uint32_t* out_err;           // [n_words][n]
    uint64_t* out_vals;          // optional [n][n_rules] result registers (Eval)
    unsigned long long* hits;    // optional [n_rules] += true pairs of this evaluation (fused hit counters)
    const uint32_t* hits_gate;   // with hits: the kernels count only while *hits_gate != 0 (set on the device
                                 // from the previous evaluation's true-pair rate; else mxp_hits_kernel counts)
    uint64_t* stats;             // optional [1] += true pairs the guard-index kernel set
    mxp_err_rec* errlog;
    uint32_t* errcount;
    mxp_ref_rec* refs;           // optional: referenced-attribute records (the *_refs kernels)
    uint32_t* refcount;
    uint32_t refcap;
    uint32_t errcap;
    uint32_t flags;              // debug / ablation: 1 = skip in-wave VM, 2 = no guards (results invalid)
    const uint32_t* fill_masks;  // mxp_fill_kernel: rules of each group of a chunk (mxp_fill.moff)
    // value classes (kernels.hip mxp_vt_*; null gvt_off: none)
    const uint32_t* gvt_off;     // [n_words + 1] merge entries of each group
    const uint32_t* gvt;         // active slot << 24 | word position j within the slot's words
    const uint32_t* gvt_mask;    // [n_words] the active slots each group's merge entries name (ascending, one each)
    const uint32_t* vt_meta;     // [n_vt][8] MXP_VTM_* fields
    const uint32_t* vt_words;    // (group, rule mask) pairs of every slot's words
    uint16_t* vt_cls;            // [n_vt][MXP_VT_PITCH(n)] class of each request
    uint32_t* vt_tm;             // class words, (match, error) u32 pairs: slot a, word j, class k at pair tbase + j * cap + k
    uint32_t* vt_cnt;            // requests of each class (mxp_vt_classify_kernel): value-class hit counters
    unsigned long long* vt_keys; // class tables: keys (MXP_VT_EMPTY = free) and a representative request
    uint32_t* vt_rep;
    uint32_t n_vt;
    uint32_t vt_imm;             // every active class table has MXP_VTI_CAP (64) slots: mxp_vtfill_imm<n_vt>_kernel
#define MXP_VTF_TILES 4u         // value-class fill: tiles of 1024 requests per workgroup
#define MXP_VTF_MARKS(n, chunks) ((((uint64_t)(n) + 1024u * MXP_VTF_TILES - 1u) / (1024u * MXP_VTF_TILES)) * (chunks) * MXP_VTF_TILES * 4u)
    uint8_t* vtf_slow;           // [fill chunk][block][MXP_VTF_TILES * 4] wave-tiles the immediate-offset fill leaves
                                 // to mxp_vtfill_imm_slow<n_vt>_kernel (the batch's vtf_slow; null: the LDS-row kernel)
    uint32_t nfa;                // some regexp of the rule set or batch is a bit-parallel NFA: the *_nfa kernels
    unsigned long long* wave_t;  // profiling (MXP_WAVE_TIMES): index kernel waves' {start, end, XCC, 5 phase marks}
    uint8_t* req_err;            // optional [n]: 1 when some rule fails for the request (compact error output)
    // Deferred true pairs (kernels.hip "Deferred pairs"; null dtp_ent / dtp_off: off).  The index
    // kernel runs before the value-class fill and records its true / error pairs per wave instead of
    // OR-ing them into rows nobody has written yet; mxp_dtp_sort_kernel files them by (fill chunk,
    // lane quad); the fill ORs them into the words it streams out.
    uint32_t* dtp_ent;           // index kernel: [waves][dtp_cap] rule | plane << 23 | lane << 24
    uint32_t* dtp_n;             // [waves] entries recorded (<= dtp_cap)
    uint32_t* dtp_ovf_n;         // [2]: overflow pairs, overflow list full (-> the gated index re-run)
    uint32_t* dtp_ovf_next;      // the other evaluation parity's [2], reset by mxp_dtp_sort_kernel
    uint32_t* dtp_ovf;           // [dtp_ovf_cap][2] (request, rule | plane << 31) past a wave's dtp_cap
                                 // or a quad's 8 slots; OR-ed in by the gated index launch after the fill
    const uint32_t* dtp_chunk;   // [n_words] value-class fill chunk << 8 | group within it (~0: none)
    uint16_t* dtp_slots;         // [chunks][tiles * 256 lane quads][8] g << 8 | plane << 7 | request % 4 << 5 | bit
    uint8_t* dtp_qn;             // [chunks][tiles * 256] entries in each quad's slots (<= 8)
    const uint32_t* dtp_gate;    // index re-run with OR-ed pairs: returns unless *dtp_gate (list full)
    uint32_t* dtp_part;          // fused hit counters of deferred pairs: [tiles][(n_rules + 1) / 2] u16
                                 // pairs, each sort workgroup's per-rule true pairs (LDS histogram),
                                 // summed into kargs.hits by mxp_dtp_hits_kernel (null: counted per pair)
    uint32_t dtp_cap, dtp_ovf_cap, dtp_tiles, dtp_nchunks;  // (chunk rows of dtp_slots / dtp_qn: MXP_DTP_ROW quads)
    uint32_t req_err_init;       // the deferred-pair index kernel writes every request's req_err flag
    uint32_t tmpl_lite;          // index templates hold no lookups / virtual columns / regexps (lite kernel)
    uint32_t* gate_out;          // the gated index launch after a counted evaluation: next gate = 0
    uint32_t dtp_t0, dtp_tn;     // mxp_dtp_sort_kernel: tiles [dtp_t0, dtp_t0 + dtp_tn) (request chunks; tn 0: all)
    uint32_t dtp_cbase;          // fill launches: chunk id of blockIdx.y 0 (plain fill chunks first, then
                                 // the value-class ones)
    uint32_t post_tmpl;
    // string heads ([n_cols][n] 16 bytes, null: none): a string value's first 12 bytes (zero past its
    // length) and its length in the last word -- the batch layout's inline view of every string
    // value, so the index kernel hashes and verifies short prefixes without the string's descriptor
    // and bytes (two dependent scattered loads per request)
    const uint4* heads;
    // a Resolve's evaluation (resolver.cpp "pair Resolve"): the plain fill stores its words only when
    // this evaluation's deferred pairs overflowed (*dtp_lazy, its dtp_ovf_n[0], nonzero) -- otherwise
    // the Resolve reads the filed pairs themselves and the match bitmap is never written (null: store)
    const uint32_t* dtp_lazy;
} mxp_kargs;

// mxp_vtd_final_kernel: the packer's provisional class tables and the candidate column of each
// active value-class slot
typedef struct mxp_vtd_final_args {
    const unsigned long long* tkey;
    const uint2* tcr;
    uint32_t cand[MXP_VT_MAX];
} mxp_vtd_final_args;
