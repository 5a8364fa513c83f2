// lower.cpp -- see lower.h.
//
// Shape-specialised lowering.  The reference VM addresses its operand stack top-relatively, and the
// reference compiler sometimes reaches a label with different stack contents on different paths
// (e.g. `ar[as] | "foo"` leaves the map `ar` behind when `as` is missing; an OR whose left operand
// ignores nmJmpOnValue leaves an extra value).  To give every stack slot a static register we lower
// each (IL address, incoming stack shape) pair -- a *context* -- separately: a label reached with two
// shapes gets two copies of the code that follows it, each with its own exact layout, so garbage
// below the top is modelled exactly as the reference sees it.  Contexts are emitted in IL-address
// order, which keeps every VM jump forward.
//
// Limits of the reference VM (interpreter.go:39-44, interpreterRun.go) are reproduced, not refused:
//   * stack: 64 u32 words.  A context's shape fixes its word count, so each push's overflow check
//     (`sp > opStackSize-k`, checked before the attribute lookup) is decided at lowering time and
//     becomes a VM_ERR "stack overflow" on exactly the paths that reach it;
//   * heap: 64 slots, `hp == heapSize-1` -> "heap overflow" after the lookup succeeded
//     (interpreterRun.go:171-172, :472, :566, :592, :698, :998, :1036, :1064, :1091, :1117); extern
//     returns skip the check (extern.go:210-237), so hp can reach 64 and the next slot write is Go's
//     "index out of range" panic.  When no path can reach slot 63 (every real rule) nothing is
//     emitted.  Otherwise the rule is lowered again: with the exact per-path count when every merge
//     agrees on it, else with the count kept in a VM register (VM_HEAP at each allocation);
//   * more than MXP_VM_MAXREG stack slots: stack slots are virtual registers; when a program has
//     more than the kernels' register file, a liveness-based colouring maps them onto it (garbage
//     slots that are never read again take no register).
#include "lower.h"

#include <algorithm>
#include <bitset>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>

#include "goutil.h"
#include "vmopt.h"
#include "../../include/mxp_batch.h"

namespace mxp {
namespace {

enum Cls : uint8_t { C_S = W_S, C_B = W_B, C_I = W_I, C_D = W_D, C_F = W_F };

constexpr size_t kMaxVmCode = 1u << 16;
constexpr size_t kMaxContexts = 1u << 14;  // (each IL instruction reached is a context)
constexpr int kStackWords = 64;  // interpreter.go:39 opStackSize
constexpr int kHeapSize = 64;    // interpreter.go:42 heapSize
constexpr int kHeapReg = 65;     // virtual register of the dynamic heap count (above every stack slot)

// Provenance of a string slot, for run-time regexp patterns: the packer compiles every value a
// pattern can take in a batch.  "c" + attr: the attribute's string values; "v" + attr + '\0' + key:
// map[key] values; "m" + attr: every value of the map; "k" + string id: a constant.
using SrcSet = std::set<std::string>;

struct Slot {
    Cls cls;
    bool konst = false;
    uint64_t kval = 0;   // register value of the constant
    std::string ktext;   // text of a constant string
    std::string attr;    // attribute the slot was resolved from (resolve_f), for fusion
    SrcSet src;          // string values it can hold (valid when !src_open)
    bool src_open = true;
};

struct State {
    std::vector<Slot> st;
    int words = 0;
    int heap = 0;
    bool heap_exact = true;  // every path into this state allocated exactly `heap` slots
};

std::string signature(const State& s, bool with_heap) {
    std::string sig;
    for (const Slot& x : s.st) sig.push_back((char)('0' + x.cls));
    if (with_heap) sig += "/" + std::to_string(s.heap);
    return sig;
}

int words_of(Cls c) { return (c == C_I || c == C_D) ? 2 : 1; }

struct Irregular {
    std::string why;
};

// merge two states of the same signature
void merge_into(State& dst, const State& src) {
    for (size_t i = 0; i < dst.st.size(); i++) {
        Slot& a = dst.st[i];
        const Slot& b = src.st[i];
        if (!(a.konst && b.konst && a.kval == b.kval && a.ktext == b.ktext)) {
            a.konst = false;
            a.ktext.clear();
        }
        if (a.attr != b.attr) a.attr.clear();
        if (a.src_open || b.src_open) {
            a.src_open = true;
            a.src.clear();
        } else {
            a.src.insert(b.src.begin(), b.src.end());
        }
    }
    if (dst.heap != src.heap || !src.heap_exact) dst.heap_exact = false;
    dst.heap = std::max(dst.heap, src.heap);
}

struct Ctx {
    State state;
    std::vector<size_t> sources;  // VM instructions whose jump target (z) is this context's block
    bool has_fallthrough = false;
};

// how the lowering treats the reference heap (see the file comment)
enum HeapMode { HM_BOUND, HM_STATIC, HM_DYNAMIC };

// registers an instruction reads / writes, over the lowering's virtual registers
using RegSet = std::bitset<128>;
RegSet vreads(const mxp_vm_ins& i) {
    RegSet r;
    switch (i.op & 0x7F) {
    case VM_EQ: case VM_LOGIC: case VM_LOOKUP: case VM_STRFN: case VM_IPEQ: case VM_TSEQ: case VM_REGEXD:
    case VM_REGEXR:
        r.set(i.a);
        r.set(i.b);
        break;
    case VM_EQK: case VM_NOT: case VM_LOGICK: case VM_JZ: case VM_JNZ: case VM_RET: case VM_LOOKUPK:
    case VM_STRFNK: case VM_IPOF: case VM_TSOF: case VM_FTOS: case VM_STOF: case VM_JZRET: case VM_JNZRET:
    case VM_MOV: case VM_REGEX:
        r.set(i.a);
        break;
    case VM_HEAP:
        r.set(i.d);
        break;
    default: break;
    }
    return r;
}
bool vwrites(const mxp_vm_ins& i) {
    switch (i.op & 0x7F) {
    case VM_RES: case VM_TRES: case VM_VCOL: case VM_CONST: case VM_EQ: case VM_EQK: case VM_NOT: case VM_LOGIC:
    case VM_LOGICK: case VM_LOOKUP: case VM_LOOKUPK: case VM_STRFN: case VM_STRFNK: case VM_IPOF: case VM_TSOF:
    case VM_IPEQ: case VM_TSEQ: case VM_FTOS: case VM_STOF: case VM_MOV: case VM_REGEX: case VM_REGEXD:
    case VM_REGEXR: case VM_HEAP:
        return true;
    default:
        return false;
    }
}
bool vterminal(const mxp_vm_ins& i) {
    const uint32_t op = i.op & 0x7F;
    return op == VM_JMP || op == VM_RET || op == VM_RETK || op == VM_ERR;
}

// Maps the virtual registers of a forward-only program onto [0, limit) by greedy colouring of the
// interference graph (a register written at pc interferes with every register live after pc).
// Returns the number of registers used, or -1 when more than `limit` are live at once (the code is
// then unchanged).
int colour_registers(std::vector<mxp_vm_ins>& code, int limit) {
    const size_t n = code.size();
    std::vector<RegSet> live_in(n + 1);
    std::vector<std::set<int>> adj(128);
    RegSet used;
    for (size_t p = n; p-- > 0;) {
        const mxp_vm_ins& i = code[p];
        RegSet out;
        if (!vterminal(i) && p + 1 < n) out |= live_in[p + 1];
        if (vm_is_jump(i) && i.z < n) out |= live_in[i.z];
        const RegSet rd = vreads(i);
        used |= rd;
        RegSet in = out;
        if (vwrites(i)) {
            const int d = i.d;
            used.set(d);
            for (int r = 0; r < 128; r++)
                if (out.test(r) && r != d) {
                    adj[d].insert(r);
                    adj[r].insert(d);
                }
            // TRES / try-LOOKUP write d only on the jump path: the fall-through keeps d's old value
            const bool partial = vm_is_jump(i);
            if (!partial) in.reset(d);
        }
        in |= rd;
        live_in[p] = in;
    }
    std::vector<int> colour(128, -1);
    int ncol = 0;
    for (int r = 0; r < 128; r++) {
        if (!used.test(r)) continue;
        uint64_t taken = 0;
        for (int s : adj[r])
            if (colour[s] >= 0) taken |= 1ull << colour[s];
        int c = 0;
        while (c < limit && (taken >> c) & 1u) c++;
        if (c >= limit) return -1;
        colour[r] = c;
        ncol = std::max(ncol, c + 1);
    }
    for (auto& i : code) {
        const RegSet rd = vreads(i);
        const uint32_t op = i.op & 0x7F;
        const bool w = vwrites(i);
        if (w || op == VM_HEAP) i.d = (uint8_t)colour[i.d];
        // a / b are register operands exactly when the op reads them
        const bool two = op == VM_EQ || op == VM_LOGIC || op == VM_LOOKUP || op == VM_STRFN || op == VM_IPEQ ||
                         op == VM_TSEQ || op == VM_REGEXD || op == VM_REGEXR;
        if (rd.any() && op != VM_HEAP) i.a = (uint8_t)colour[i.a];
        if (two) i.b = (uint8_t)colour[i.b];
    }
    return ncol;
}

class Lowerer {
  public:
    Lowerer(const IlProgram& p, LowerTables* t, HeapMode hm) : p_(p), t_(t), hm_(hm) {}

    LoweredRule run() {
        LoweredRule out;
        const IlFunction* f = p_.get("eval");
        if (!f) {
            out.why = "no eval function";
            return out;
        }
        fn_ret_ = f->ret;
        try {
            body(*f);
            finish();
        } catch (Irregular& ir) {
            out.why = ir.why;
            return out;
        }
        out.ok = true;
        out.code = code_;
        out.nregs = maxregs_;
        out.uses_ipof = ipof_;
        out.uses_rxof = rxof_;
        out.uses_tsof = tsof_;
        out.uses_strings = strings_;
        out.uses_maps = maps_;
        return out;
    }

    bool heap_risk() const { return heap_risk_; }
    bool heap_inexact() const { return heap_inexact_; }

  private:
    // ------------------------------------------------------------------ emission helpers
    size_t emit(uint8_t op, int d, int a, int b, uint32_t x, uint32_t y, uint32_t z) {
        if (code_.size() >= kMaxVmCode) throw Irregular{"lowered program too large"};
        mxp_vm_ins i;
        i.op = op;
        i.d = (uint8_t)d;
        i.a = (uint8_t)a;
        i.b = (uint8_t)b;
        i.x = x;
        i.y = y;
        i.z = z;
        code_.push_back(i);
        return code_.size() - 1;
    }

    int top() const { return (int)cur_.st.size() - 1; }

    Slot& push(Cls c) {
        Slot s;
        s.cls = c;
        cur_.st.push_back(s);
        cur_.words += words_of(c);
        // the callers checked the reference's overflow condition first (room())
        if (cur_.words > kStackWords) throw Irregular{"internal: stack past 64 words"};
        maxregs_ = std::max<uint32_t>(maxregs_, (uint32_t)cur_.st.size());
        return cur_.st.back();
    }

    Slot pop_raw() {
        if (cur_.st.empty()) throw Irregular{"stack underflow"};
        Slot s = cur_.st.back();
        cur_.st.pop_back();
        cur_.words -= words_of(s.cls);
        return s;
    }

    // Pop an operand the reference reads as `want`.  A string read from a slot that holds an
    // interface value is Go's `heap[i].(string)` (emulated by VM_FTOS); interface reads of a string
    // slot just see the string.  Other mismatches would reinterpret raw words: not lowered.
    Slot pop(Cls want) {
        if (cur_.st.empty()) throw Irregular{"stack underflow"};
        Slot s = cur_.st.back();
        int reg = top();
        if (s.cls != want) {
            if (want == C_S && s.cls == C_F) {
                emit(VM_FTOS, reg, reg, 0, 0, 0, 0);
                s.cls = C_S;
                s.konst = false;
            } else if (want == C_F && s.cls == C_S) {
                emit(VM_STOF, reg, reg, 0, 0, 0, 0);
                s.cls = C_F;
                s.konst = false;
            } else {
                throw Irregular{"operand type mismatch"};
            }
        }
        pop_raw();
        return s;
    }

    // The reference checks operand availability before touching anything (interpreterRun.go, e.g.
    // :247 `if sp < 2 goto STACK_UNDERFLOW`).  Paths of an OR chain can reach a consumer with too few
    // values; those paths raise "stack underflow" there.
    bool need(size_t k) {
        if (cur_.st.size() >= k) return true;
        emit(VM_ERR, 0, 0, 0, 0, ERR_UNDERFLOW, 0);
        live_ = false;
        return false;
    }

    // The reference's overflow check of a push (`if sp > opStackSize-k goto STACK_OVERFLOW`, made
    // before the lookup): k words must fit.  Paths that fail it raise "stack overflow" here.
    bool room(int k) {
        if (cur_.words + k <= kStackWords) return true;
        emit(VM_ERR, 0, 0, 0, 0, ERR_OVERFLOW, 0);
        live_ = false;
        return false;
    }

    // One heap allocation at the current point of the path.  `checked`: the reference tests
    // `hp == heapSize-1` first (resolve / push / lookup); extern returns do not.  Returns false when
    // the path ends here (overflow error or index panic emitted).
    bool alloc(bool checked) {
        switch (hm_) {
        case HM_BOUND:
            // first pass: an upper bound of the count; a rule whose bound reaches slot 63 is lowered
            // again with the exact count (run_lowering)
            if (cur_.heap >= kHeapSize - 1) heap_risk_ = true;
            cur_.heap++;
            return true;
        case HM_STATIC:
            if (checked && cur_.heap == kHeapSize - 1) {
                emit(VM_ERR, 0, 0, 0, 0, ERR_HEAP, 0);
                live_ = false;
                return false;
            }
            if (cur_.heap >= kHeapSize) {
                emit(VM_ERR, 0, 0, 0, 0, PANIC_INDEX, 0);
                live_ = false;
                return false;
            }
            cur_.heap++;
            return true;
        case HM_DYNAMIC:
            emit(VM_HEAP, kHeapReg, 0, 0, 0, checked ? 1u : 0u, 0);
            return true;
        }
        return true;
    }

    void add_edge(uint32_t target, const State& s, size_t vm_src, bool fallthrough) {
        if (target <= at_ && !fallthrough) throw Irregular{"backward jump"};
        std::string sig = signature(s, hm_ == HM_STATIC);
        auto& bucket = pending_[target];
        auto it = bucket.find(sig);
        if (it == bucket.end()) {
            if (++ncontexts_ > kMaxContexts) throw Irregular{"too many stack-shape contexts"};
            Ctx c;
            c.state = s;
            it = bucket.emplace(sig, c).first;
            order_[target].push_back(sig);
        } else {
            merge_into(it->second.state, s);
            if (!it->second.state.heap_exact) heap_inexact_ = true;
        }
        if (fallthrough) it->second.has_fallthrough = true;
        else it->second.sources.push_back(vm_src);
    }

    std::string str(uint32_t id) const { return p_.strings.get(id); }

    static Cls want_of_resolve(uint32_t op) {
        switch (op) {
        case ResolveS: case TResolveS: return C_S;
        case ResolveB: case TResolveB: return C_B;
        case ResolveI: case TResolveI: return C_I;
        case ResolveD: case TResolveD: return C_D;
        default: return C_F;
        }
    }

    // words the reference's overflow check of a resolve needs (interpreterRun.go:455-708: note that
    // resolve_f checks for two words although it pushes one)
    static int resolve_room(uint32_t op) {
        switch (op) {
        case ResolveS: case ResolveB: return 1;
        case ResolveI: case ResolveD: case ResolveF: return 2;
        case TResolveS: case TResolveB: case TResolveF: return 2;
        default: return 3;  // TResolveI / TResolveD
        }
    }

    bool is_target(uint32_t addr) const { return jump_targets_.count(addr) != 0; }

    static void set_src(Slot& s, const std::string& src) {
        s.src.clear();
        s.src.insert(src);
        s.src_open = false;
    }
    std::string const_src(uint32_t sid) const { return "k" + std::to_string(sid); }

    // a string slot holding map lookups of `m` (const key or not); `missing_empty`: "" when absent
    void lookup_src(Slot& dst, const Slot& m, const std::string* key, bool missing_empty) {
        dst.src.clear();
        dst.src_open = m.src_open;
        if (m.src_open) return;
        for (const std::string& s : m.src) {
            if (s.empty() || s[0] != 'c') {  // a map that is not an attribute value
                dst.src_open = true;
                dst.src.clear();
                return;
            }
            dst.src.insert(key ? "v" + s.substr(1) + std::string(1, '\0') + *key : "m" + s.substr(1));
        }
        if (missing_empty) dst.src.insert(const_src(t_->intern_string("")));
    }

    // ------------------------------------------------------------------ driver
    void body(const IlFunction& f) {
        const auto& c = p_.code;
        start_ = f.address;
        end_ = f.address + f.length;
        // every address some jump names (fused pairs must not be split by a jump)
        for (uint32_t a = start_; a < end_;) {
            const OpInfo* inf = op_info(c[a]);
            if (!inf) throw Irregular{"unknown opcode"};
            if (c[a] == Jmp || c[a] == Jz || c[a] == Jnz) jump_targets_.insert(c[a + 1]);
            a += op_words(c[a]);
        }
        if (hm_ == HM_DYNAMIC) emit(VM_CONST, kHeapReg, 0, 0, 0, 0, 0);  // hp = 0
        Ctx entry;
        entry.has_fallthrough = true;
        const std::string sig0 = signature(entry.state, hm_ == HM_STATIC);
        pending_[start_].emplace(sig0, entry);
        order_[start_].push_back(sig0);
        ncontexts_ = 1;
        // A fall-through edge into a context is honoured only if that context's block is emitted
        // immediately after its predecessor; otherwise an explicit VM_JMP is appended (prev_ctx_).
        for (uint32_t a = start_; a < end_;) {
            uint32_t sz = op_words(c[a]);
            auto pit = pending_.find(a);
            if (pit != pending_.end()) {
                for (const std::string& sig : order_[a]) {
                    Ctx& cx = pit->second.at(sig);
                    block(a, cx);
                }
                pending_.erase(pit);
            }
            a += sz;
        }
        if (!pending_.empty()) throw Irregular{"jump outside function"};
    }

    // Lower the instruction(s) at `a` for one incoming context.
    void block(uint32_t a, Ctx& cx) {
        at_ = a;
        cur_ = cx.state;
        size_t start_index = code_.size();
        const std::string sig = signature(cur_, hm_ == HM_STATIC);
        // patch jumps into this block
        for (size_t s : cx.sources) code_[s].z = (uint32_t)start_index;
        for (size_t s : pending_ft_jumps_[{a, sig}]) code_[s].z = (uint32_t)start_index;
        wake_.insert(start_index);
        uint32_t next = lower_one(a);
        // fall-through successor
        if (live_) {
            State s = cur_;
            add_edge(next, s, 0, true);
            // emit an explicit jump; removed later when it lands on the next instruction
            size_t j = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
            pending_ft_jumps_[{next, signature(s, hm_ == HM_STATIC)}].push_back(j);
        }
        if (code_.size() == start_index) emit(VM_NOP, 0, 0, 0, 0, 0, 0);
    }

    // Lowers the instruction at `a` (plus a fused successor) from cur_; returns the next address.
    // Sets live_ = false when control does not fall through.
    uint32_t lower_one(uint32_t a) {
        const auto& c = p_.code;
        uint32_t op = c[a];
        const OpInfo* inf = op_info(op);
        uint32_t next = a + op_words(op);
        live_ = true;
        switch (op) {
        case ResolveS: case ResolveB: case ResolveI: case ResolveD: case ResolveF: {
            Cls w = want_of_resolve(op);
            std::string attr = str(c[a + 1]);
            if (!room(resolve_room(op))) return next;
            // fuse `resolve_f <map>; anlookup "k"` into a virtual column (not when the rule's heap
            // is tracked exactly: the two allocations may fail between the lookups)
            if (op == ResolveF && next < end_ && c[next] == ANLookup && !is_target(next) &&
                t_->attr_type(attr) == VT_STRING_MAP && hm_ == HM_BOUND) {
                std::string key = str(c[next + 1]);
                const uint32_t vc = t_->vcolumn(attr, key);
                Slot& s = push(C_S);
                set_src(s, "v" + attr + std::string(1, '\0') + key);
                alloc(true);
                alloc(true);
                emit(VM_VCOL, top(), 0, 0, vc, 0, t_->intern_string(attr));
                return next + op_words(ANLookup);
            }
            {
                Slot& s = push(w);
                s.attr = attr;
                if (w == C_S || w == C_F) set_src(s, "c" + attr);
            }
            emit(VM_RES, top(), 0, 0, t_->column(attr), w, t_->intern_string(attr));
            if (w == C_S || w == C_F) alloc(true);
            return next;
        }
        case TResolveS: case TResolveB: case TResolveI: case TResolveD: case TResolveF: {
            if (next >= end_ || c[next] != Jnz || is_target(next)) throw Irregular{"tresolve not followed by a private jnz"};
            Cls w = want_of_resolve(op);
            std::string attr = str(c[a + 1]);
            const uint32_t after = next + op_words(Jnz);
            if (!room(resolve_room(op))) return after;
            State saved = cur_;
            {
                Slot& s = push(w);
                s.attr = attr;
                if (w == C_S || w == C_F) set_src(s, "c" + attr);
            }
            const bool allocs = w == C_S || w == C_F;
            int reg = top();
            if (allocs && hm_ != HM_BOUND) {
                // found -> allocation (may fail) -> jump target; not found -> fall through
                State found = cur_;
                size_t j = emit(VM_TRES, reg, 0, 0, t_->column(attr), w, 0);
                size_t jn = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
                add_edge(after, saved, jn, false);
                code_[j].z = (uint32_t)code_.size();
                cur_ = found;
                if (alloc(true)) {
                    size_t jf = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
                    add_edge(c[next + 1], cur_, jf, false);
                }
                live_ = false;
                return after;
            }
            if (allocs) alloc(true);
            State found = cur_;
            cur_ = saved;
            size_t j = emit(VM_TRES, reg, 0, 0, t_->column(attr), w, 0);
            add_edge(c[next + 1], found, j, false);
            return after;
        }
        case APushS: {
            if (!room(1)) return next;
            if (!alloc(true)) return next;
            Slot& s = push(C_S);
            std::string txt = str(c[a + 1]);
            uint32_t id = t_->intern_string(txt);
            s.konst = true;
            s.kval = id;
            s.ktext = txt;
            set_src(s, const_src(id));
            emit(VM_CONST, top(), 0, 0, 0, id, 0);
            return next;
        }
        case APushB: {
            if (!room(1)) return next;
            Slot& s = push(C_B);
            s.konst = true;
            s.kval = c[a + 1];
            emit(VM_CONST, top(), 0, 0, 0, c[a + 1], 0);
            return next;
        }
        case APushI: case APushD: {
            if (!room(2)) return next;
            uint64_t v = (uint64_t)c[a + 1] | ((uint64_t)c[a + 2] << 32);
            Slot& s = push(op == APushI ? C_I : C_D);
            s.konst = true;
            s.kval = v;
            emit(VM_CONST, top(), 0, 0, 0, (uint32_t)v, (uint32_t)(v >> 32));
            return next;
        }
        case EqS: case EqB: case EqI: case EqD: {
            Cls k = op == EqS ? C_S : op == EqB ? C_B : op == EqI ? C_I : C_D;
            if (!need(2)) return next;
            pop(k);
            pop(k);
            push(C_B);
            emit(VM_EQ, top(), top(), top() + 1, 0, 0, 0);
            return next;
        }
        case AEqS: {
            if (!need(1)) return next;
            pop(C_S);
            push(C_B);
            emit(VM_EQK, top(), top(), 0, 0, t_->intern_string(str(c[a + 1])), 0);
            return next;
        }
        case AEqB: case AEqI: case AEqD: {
            if (!need(1)) return next;
            Cls k = op == AEqB ? C_B : op == AEqI ? C_I : C_D;
            pop(k);
            push(C_B);
            emit(VM_EQK, top(), top(), 0, 0, c[a + 1], op == AEqB ? 0 : c[a + 2]);
            return next;
        }
        case Not:
            if (!need(1)) return next;
            pop(C_B);
            push(C_B);
            emit(VM_NOT, top(), top(), 0, 0, 0, 0);
            return next;
        case And: case Or: case Xor:
            if (!need(2)) return next;
            pop(C_B);
            pop(C_B);
            push(C_B);
            emit(VM_LOGIC, top(), top(), top() + 1, 0, op == And ? 0 : op == Or ? 1 : 2, 0);
            return next;
        case AAnd: case AOr: case AXor:
            if (!need(1)) return next;
            pop(C_B);
            push(C_B);
            emit(VM_LOGICK, top(), top(), 0, c[a + 1], op == AAnd ? 0 : op == AOr ? 1 : 2, 0);
            return next;
        case Jz: case Jnz: {
            if (!need(1)) return next;
            pop(C_B);
            size_t j = emit(op == Jz ? VM_JZ : VM_JNZ, 0, top() + 1, 0, 0, 0, 0);
            add_edge(c[a + 1], cur_, j, false);
            return next;
        }
        case Jmp: {
            size_t j = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
            add_edge(c[a + 1], cur_, j, false);
            live_ = false;
            return next;
        }
        case Ret: {
            Cls want = fn_ret_ == IL_BOOL ? C_B : fn_ret_ == IL_STRING ? C_S
                       : (fn_ret_ == IL_INTEGER || fn_ret_ == IL_DURATION) ? C_I
                       : fn_ret_ == IL_DOUBLE ? C_D : C_F;
            if (!need(1)) return next;
            Slot s = pop(want);
            (void)s;
            emit(VM_RET, 0, top() + 1, 0, 0, fn_ret_ == IL_BOOL ? 1 : 0, fn_ret_);
            live_ = false;
            return next;
        }
        case ANLookup: case ALookup: {
            if (!need(1)) return next;
            Slot m = pop(C_F);
            const std::string key = str(c[a + 1]);
            Slot& s = push(C_S);
            lookup_src(s, m, &key, op == ANLookup);
            maps_ = true;
            emit(VM_LOOKUPK, top(), top(), 0, t_->intern_string(key), op == ANLookup ? LK_N : LK_ERR, 0);
            alloc(true);
            return next;
        }
        case NLookup: case Lookup: {
            if (!need(2)) return next;
            Slot k = pop(C_S);
            Slot m = pop(C_F);
            Slot& s = push(C_S);
            lookup_src(s, m, k.konst ? &k.ktext : nullptr, op == NLookup);
            maps_ = true;
            emit(VM_LOOKUP, top(), top(), top() + 1, 0, op == NLookup ? LK_N : LK_ERR, 0);
            alloc(true);
            return next;
        }
        case TLookup: {
            if (next >= end_ || c[next] != Jnz || is_target(next)) throw Irregular{"tlookup not followed by a private jnz"};
            const uint32_t after = next + op_words(Jnz);
            if (!need(2)) return after;
            Slot k = pop(C_S);
            Slot m = pop(C_F);
            State saved = cur_;
            {
                Slot& s = push(C_S);
                lookup_src(s, m, k.konst ? &k.ktext : nullptr, false);
            }
            int reg = top();
            maps_ = true;
            if (hm_ != HM_BOUND) {
                State found = cur_;
                size_t j = emit(VM_LOOKUP, reg, reg, reg + 1, 0, LK_TRY, 0);
                size_t jn = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
                add_edge(after, saved, jn, false);
                code_[j].z = (uint32_t)code_.size();
                cur_ = found;
                if (alloc(true)) {
                    size_t jf = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
                    add_edge(c[next + 1], cur_, jf, false);
                }
                live_ = false;
                return after;
            }
            alloc(true);
            State found = cur_;
            cur_ = saved;
            size_t j = emit(VM_LOOKUP, reg, reg, reg + 1, 0, LK_TRY, 0);
            add_edge(c[next + 1], found, j, false);
            return after;
        }
        case Call:
            call(str(c[a + 1]));
            return next;
        default:
            throw Irregular{std::string("opcode not lowered: ") + (inf ? inf->keyword : "?")};
        }
    }

    void call(const std::string& name) {
        if (name == "ip" || name == "timestamp") {
            if (!need(1)) return;
            // interpreterRun.go:899-900 write two result words at sp-1 and sp: at sp == 64 the
            // second is past the 64-word stack (Go's index panic), after the extern returned
            const bool past_stack = cur_.words == kStackWords;
            Slot s = pop(C_S);
            push(C_F);
            bool ip = name == "ip";
            if (s.konst) {
                const std::string& txt = s.ktext;
                if (ip) {
                    uint8_t b[16];
                    if (go_parse_ip((const uint8_t*)txt.data(), txt.size(), b)) {
                        uint64_t h = MXP_FH(MXP_BYTES, t_->intern_bytes(std::string((const char*)b, 16)));
                        emit(VM_CONST, top(), 0, 0, 0, (uint32_t)h, (uint32_t)(h >> 32));
                    } else {
                        emit(VM_ERR, top(), 0, 0, 0, ERR_IP, (uint32_t)s.kval);
                        live_ = false;
                        return;
                    }
                } else {
                    int64_t sec;
                    int32_t ns;
                    if (go_parse_rfc3339((const uint8_t*)txt.data(), txt.size(), &sec, &ns)) {
                        uint64_t h = MXP_FH(MXP_TIMESTAMP, t_->intern_time(sec, ns));
                        emit(VM_CONST, top(), 0, 0, 0, (uint32_t)h, (uint32_t)(h >> 32));
                    } else {
                        emit(VM_ERR, top(), 0, 0, 0, ERR_TS, (uint32_t)s.kval);
                        live_ = false;
                        return;
                    }
                }
            } else {
                if (ip) ipof_ = true;
                else tsof_ = true;
                emit(ip ? VM_IPOF : VM_TSOF, top(), top(), 0, 0, 0, 0);
            }
            // the extern's interface result takes a heap slot without the overflow check
            // (extern.go:232-237); then the result words are stored
            if (!alloc(false)) return;
            if (past_stack) {
                emit(VM_ERR, 0, 0, 0, 0, PANIC_INDEX, 0);
                live_ = false;
            }
            return;
        }
        if (name == "ip_equal" || name == "timestamp_equal") {
            if (!need(2)) return;
            pop(C_F);
            pop(C_F);
            push(C_B);
            emit(name == "ip_equal" ? VM_IPEQ : VM_TSEQ, top(), top(), top() + 1, 0, 0, 0);
            return;
        }
        int fn = name == "match" ? SF_MATCH : name == "startsWith" ? SF_STARTS : name == "endsWith" ? SF_ENDS
                 : name == "matches" ? SF_REGEX : -1;
        if (fn < 0) throw Irregular{"call of unknown function " + name};
        if (!need(2)) return;
        Slot b = pop(C_S);
        Slot a = pop(C_S);
        push(C_B);
        if (fn == SF_REGEX) {  // externMatches(pattern = receiver, subject): regexp.MatchString
            if (a.konst) {
                std::string e;
                const int32_t id = t_->regex_const(a.ktext, &e);
                if (id == -2) throw Irregular{"regexp: " + e};
                if (id < 0) {
                    emit(VM_ERR, top(), 0, 0, 0, ERR_REGEX, (uint32_t)a.kval);
                    live_ = false;
                    return;
                }
                if (b.konst) {
                    emit(VM_CONST, top(), 0, 0, 0, t_->regex_const_match(id, b.ktext) ? 1 : 0, 0);
                    return;
                }
                strings_ = true;
                emit(VM_REGEX, top(), top() + 1, 0, (uint32_t)id, 0, 0);
                return;
            }
            // run-time pattern (externs.go:118-120 compiles it on every call): every value it can
            // take in a batch -- attribute values, map values, constants merged in by `|` -- is
            // compiled once per batch by the packer (rxof[pattern string id])
            if (a.src_open || a.src.empty()) throw Irregular{"regexp pattern of unknown provenance"};
            for (const std::string& s : a.src) {
                if (s[0] == 'k') {
                    t_->regex_source(RX_SRC_CONST, "", "", (uint32_t)std::stoul(s.substr(1)));
                } else if (s[0] == 'c') {
                    t_->regex_source(RX_SRC_COLUMN, s.substr(1), "", 0);
                } else if (s[0] == 'm') {
                    t_->regex_source(RX_SRC_MAPVALS, s.substr(1), "", 0);
                } else {  // 'v': attr '\0' key
                    const size_t z = s.find('\0');
                    t_->regex_source(RX_SRC_VCOLUMN, s.substr(1, z - 1), s.substr(z + 1), 0);
                }
            }
            strings_ = true;
            rxof_ = true;
            emit(VM_REGEXD, top(), top(), top() + 1, 0, 0, 0);
            return;
        }
        if (a.konst && b.konst) {
            const std::string& s = a.ktext;
            const std::string& q = b.ktext;
            bool r;
            if (fn == SF_STARTS) r = s.size() >= q.size() && s.compare(0, q.size(), q) == 0;
            else if (fn == SF_ENDS) r = s.size() >= q.size() && s.compare(s.size() - q.size(), q.size(), q) == 0;
            else if (!q.empty() && q.back() == '*')
                r = s.size() >= q.size() - 1 && s.compare(0, q.size() - 1, q, 0, q.size() - 1) == 0;
            else if (!q.empty() && q[0] == '*')
                r = s.size() >= q.size() - 1 && s.compare(s.size() - (q.size() - 1), q.size() - 1, q, 1, q.size() - 1) == 0;
            else r = s == q;
            emit(VM_CONST, top(), 0, 0, 0, r ? 1 : 0, 0);
            return;
        }
        strings_ = true;
        if (b.konst) emit(VM_STRFNK, top(), top(), 0, (uint32_t)b.kval, (uint32_t)fn, 0);
        else emit(VM_STRFN, top(), top(), top() + 1, 0, (uint32_t)fn, 0);
    }

    // Drop explicit fall-through jumps that land on the next instruction, renumber, set WAKE flags.
    void finish() {
        std::vector<uint32_t> newidx(code_.size() + 1, 0);
        std::vector<bool> keep(code_.size(), true);
        for (size_t i = 0; i < code_.size(); i++)
            if ((code_[i].op & 0x7F) == VM_JMP && code_[i].z == i + 1) keep[i] = false;
        uint32_t k = 0;
        for (size_t i = 0; i < code_.size(); i++) {
            newidx[i] = k;
            if (keep[i]) k++;
        }
        newidx[code_.size()] = k;
        std::vector<mxp_vm_ins> out;
        out.reserve(k);
        std::set<uint32_t> targets;
        for (size_t i = 0; i < code_.size(); i++) {
            if (!keep[i]) continue;
            mxp_vm_ins ins = code_[i];
            if (vm_is_jump(ins)) {
                if (ins.z >= code_.size()) throw Irregular{"dangling jump"};
                ins.z = newidx[ins.z];
                targets.insert(ins.z);
            }
            out.push_back(ins);
        }
        for (uint32_t t : targets) {
            if (t >= out.size()) throw Irregular{"jump past end"};
            out[t].op |= MXP_VM_WAKE;
        }
        for (size_t i = 0; i < out.size(); i++)
            if (vm_is_jump(out[i]) && out[i].z <= i) throw Irregular{"non-forward jump after layout"};
        code_ = out;
        // more stack slots than the hot kernels' register file, or the heap count register:
        // colour onto MXP_VM_MAXREG registers, else onto the deep kernels' MXP_VM_DEEPREG
        if (maxregs_ > MXP_VM_MAXREG || hm_ == HM_DYNAMIC) {
            int n = colour_registers(code_, MXP_VM_MAXREG);
            if (n < 0) n = colour_registers(code_, MXP_VM_DEEPREG);
            if (n < 0) throw Irregular{"more than MXP_VM_DEEPREG values live at once"};
            maxregs_ = (uint32_t)n;
        }
        try {
            optimize_vm(code_);
        } catch (std::exception& e) {
            throw Irregular{e.what()};
        }
    }

    const IlProgram& p_;
    LowerTables* t_;
    HeapMode hm_;
    uint8_t fn_ret_ = IL_BOOL;
    uint32_t start_ = 0, end_ = 0, at_ = 0;
    State cur_;
    bool live_ = true;
    bool heap_risk_ = false, heap_inexact_ = false;
    std::map<uint32_t, std::map<std::string, Ctx>> pending_;
    std::map<uint32_t, std::vector<std::string>> order_;
    std::map<std::pair<uint32_t, std::string>, std::vector<size_t>> pending_ft_jumps_;
    std::set<uint32_t> jump_targets_;
    std::set<size_t> wake_;
    size_t ncontexts_ = 0;
    std::vector<mxp_vm_ins> code_;
    uint32_t maxregs_ = 0;
    bool ipof_ = false, tsof_ = false, strings_ = false, maps_ = false, rxof_ = false;
};

}  // namespace

LoweredRule lower_rule(const IlProgram& prog, LowerTables* tables) {
    // pass 1 bounds the heap count; a rule whose bound can reach the reference's overflow slot is
    // lowered again with the exact count -- statically when every merge agrees on it
    Lowerer bound(prog, tables, HM_BOUND);
    LoweredRule r = bound.run();
    if (!r.ok || !bound.heap_risk()) return r;
    Lowerer exact(prog, tables, bound.heap_inexact() ? HM_DYNAMIC : HM_STATIC);
    LoweredRule e = exact.run();
    if (!e.ok && !bound.heap_inexact()) {
        // per-path contexts ran out of room: keep the count in a register instead
        Lowerer dyn(prog, tables, HM_DYNAMIC);
        e = dyn.run();
    }
    return e;
}

std::string vm_disasm(const std::vector<mxp_vm_ins>& code) {
    static const char* names[] = {"nop", "res", "tres", "vcol", "const", "eq", "eqk", "not", "jz", "jnz", "jmp",
                                  "ret", "lookup", "lookupk", "strfn", "strfnk", "ipof", "tsof", "ipeq", "tseq",
                                  "err", "logic", "logick", "ftos", "stof", "jzret", "jnzret", "retk", "mov", "regex", "regexd", "regexr",
                                  "heap"};
    std::string o;
    char buf[160];
    for (size_t i = 0; i < code.size(); i++) {
        const mxp_vm_ins& c = code[i];
        unsigned op = c.op & 0x7F;
        snprintf(buf, sizeof buf, "%3zu%s %-7s d=%u a=%u b=%u x=%u y=%u z=%u\n", i, (c.op & MXP_VM_WAKE) ? "*" : " ",
                 op < sizeof(names) / sizeof(names[0]) ? names[op] : "?", c.d, c.a, c.b, c.x, c.y, c.z);
        o += buf;
    }
    return o;
}

}  // namespace mxp
