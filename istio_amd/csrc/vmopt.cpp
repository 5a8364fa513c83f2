// vmopt.cpp -- see vmopt.h.
#include "vmopt.h"

#include <cstdint>
#include <stdexcept>

namespace mxp {

static inline uint32_t opof(const mxp_vm_ins& i) { return i.op & 0x7Fu; }

bool vm_is_jump(const mxp_vm_ins& i) {
    uint32_t op = opof(i);
    return op == VM_JMP || op == VM_JZ || op == VM_JNZ || op == VM_TRES ||
           ((op == VM_LOOKUP || op == VM_LOOKUPK) && i.y == LK_TRY);
}

static bool is_terminal(const mxp_vm_ins& i) {
    uint32_t op = opof(i);
    return op == VM_JMP || op == VM_RET || op == VM_RETK || op == VM_ERR;
}

// registers read / written (bit masks)
static uint64_t reads(const mxp_vm_ins& i) {
    switch (opof(i)) {
    case VM_EQ: case VM_LOGIC: case VM_LOOKUP: case VM_STRFN: case VM_IPEQ: case VM_TSEQ: case VM_REGEXD:
    case VM_REGEXR:
        return (1ull << i.a) | (1ull << i.b);
    case VM_EQK: case VM_NOT: case VM_LOGICK: case VM_JZ: case VM_JNZ: case VM_RET: case VM_LOOKUPK:
    case VM_STRFNK: case VM_IPOF: case VM_TSOF: case VM_FTOS: case VM_STOF: case VM_JZRET: case VM_JNZRET:
    case VM_MOV: case VM_REGEX:
        return 1ull << i.a;
    case VM_HEAP:
        return 1ull << i.d;
    default:
        return 0;
    }
}

static uint64_t writes(const mxp_vm_ins& i) {
    switch (opof(i)) {
    case VM_RES: case VM_TRES: case VM_VCOL: case VM_CONST: case VM_EQ: case VM_EQK: case VM_NOT: case VM_LOGIC:
    case VM_LOGICK: case VM_LOOKUP: case VM_LOOKUPK: case VM_STRFN: case VM_STRFNK: case VM_IPOF: case VM_TSOF:
    case VM_IPEQ: case VM_TSEQ: case VM_FTOS: case VM_STOF: case VM_MOV: case VM_REGEX: case VM_REGEXD:
    case VM_REGEXR: case VM_HEAP:
        return 1ull << i.d;
    default:
        return 0;
    }
}

// no side effects (cannot raise, cannot jump): removable when its result is dead
static bool is_pure(const mxp_vm_ins& i) {
    switch (opof(i)) {
    case VM_CONST: case VM_EQ: case VM_EQK: case VM_NOT: case VM_LOGIC: case VM_LOGICK: case VM_STRFN:
    case VM_STRFNK: case VM_STOF: case VM_NOP: case VM_MOV: case VM_REGEX: case VM_REGEXR:
        return true;
    default:
        return false;
    }
}

// Deterministic bool result of executing from pc with every register unknown, or -1.
static int det_result(const std::vector<mxp_vm_ins>& c, size_t pc) {
    bool known[MXP_VM_DEEPREG] = {false};
    uint64_t val[MXP_VM_DEEPREG] = {0};
    for (int steps = 0; steps < 64 && pc < c.size(); steps++) {
        const mxp_vm_ins& i = c[pc];
        switch (opof(i)) {
        case VM_NOP: pc++; break;
        case VM_CONST:
            known[i.d] = true;
            val[i.d] = (uint64_t)i.y | ((uint64_t)i.z << 32);
            pc++;
            break;
        case VM_NOT:
            known[i.d] = known[i.a];
            val[i.d] = val[i.a] == 0;
            pc++;
            break;
        case VM_EQK:
            known[i.d] = known[i.a];
            val[i.d] = val[i.a] == ((uint64_t)i.y | ((uint64_t)i.z << 32));
            pc++;
            break;
        case VM_EQ:
            known[i.d] = known[i.a] && known[i.b];
            val[i.d] = val[i.a] == val[i.b];
            pc++;
            break;
        case VM_LOGIC: case VM_LOGICK: {
            bool kb = opof(i) == VM_LOGIC ? known[i.b] : true;
            uint64_t q = opof(i) == VM_LOGIC ? val[i.b] : i.x;
            bool p = (uint32_t)val[i.a] != 0, r = (uint32_t)q != 0;
            known[i.d] = known[i.a] && kb;
            val[i.d] = i.y == 0 ? (p && r) : i.y == 1 ? (p || r) : (p != r);
            pc++;
            break;
        }
        case VM_STRFN: case VM_STRFNK: case VM_STOF: case VM_REGEX:
            known[i.d] = false;
            pc++;
            break;
        case VM_JZ: case VM_JNZ:
            if (!known[i.a]) return -1;
            if (((uint32_t)val[i.a] == 0) == (opof(i) == VM_JZ)) pc = i.z;
            else pc++;
            break;
        case VM_JZRET: case VM_JNZRET:
            if (!known[i.a]) return -1;
            if (((uint32_t)val[i.a] == 0) == (opof(i) == VM_JZRET)) return (int)i.y;
            pc++;
            break;
        case VM_JMP: pc = i.z; break;
        case VM_RETK: return (int)i.y;
        case VM_RET:
            if (i.y != 1 || !known[i.a]) return -1;
            return (uint32_t)val[i.a] != 0 ? 1 : 0;
        default:
            return -1;  // loads, lookups, externs: side effects or unknown data
        }
    }
    return -1;
}

static void relayout(std::vector<mxp_vm_ins>& c, const std::vector<bool>& keep) {
    std::vector<uint32_t> idx(c.size() + 1, 0);
    uint32_t k = 0;
    for (size_t i = 0; i < c.size(); i++) {
        idx[i] = k;
        if (keep[i]) k++;
    }
    idx[c.size()] = k;
    std::vector<mxp_vm_ins> out;
    out.reserve(k);
    for (size_t i = 0; i < c.size(); i++) {
        if (!keep[i]) continue;
        mxp_vm_ins ins = c[i];
        ins.op &= 0x7F;
        if (vm_is_jump(ins)) {
            // a removed target forwards to the next kept instruction (only NOPs / dead code removed)
            ins.z = idx[ins.z];
        }
        out.push_back(ins);
    }
    for (auto& ins : out)
        if (vm_is_jump(ins)) out.at(ins.z).op |= MXP_VM_WAKE;
    c.swap(out);
}

static void optimize_once(std::vector<mxp_vm_ins>& c) {
    const size_t n = c.size();
    if (n == 0) return;
    for (auto& i : c) i.op &= 0x7F;
    // 1. jump threading through unconditional jumps
    for (auto& i : c) {
        if (!vm_is_jump(i)) continue;
        for (int guard = 0; guard < 64 && opof(c[i.z]) == VM_JMP; guard++) i.z = c[i.z].z;
    }
    // 2. constant-result folding
    std::vector<int> det(n, -1);
    for (size_t p = n; p-- > 0;) det[p] = det_result(c, p);
    for (size_t p = 0; p < n; p++) {
        mxp_vm_ins& i = c[p];
        uint32_t op = opof(i);
        if ((op == VM_JZ || op == VM_JNZ || op == VM_JMP) && det[i.z] >= 0) {
            int r = det[i.z];
            if (op == VM_JMP) {
                i = mxp_vm_ins{(uint8_t)VM_RETK, 0, 0, 0, 0, (uint32_t)r, 0};
            } else {
                i.op = op == VM_JZ ? VM_JZRET : VM_JNZRET;
                i.y = (uint32_t)r;
                i.z = 0;
            }
        }
    }
    for (size_t p = 0; p < n; p++)
        if (det[p] >= 0 && opof(c[p]) != VM_RETK) c[p] = mxp_vm_ins{(uint8_t)VM_RETK, 0, 0, 0, 0, (uint32_t)det[p], 0};
    // `JZ a -> p+2 ; RETK y` == `JNZRET a, y ; (fall through to p+2)` (and symmetrically for JNZ);
    // the RETK then stays only for other jumps that land on it
    for (size_t p = 0; p + 2 < n; p++) {
        mxp_vm_ins& i = c[p];
        uint32_t op = opof(i);
        if ((op == VM_JZ || op == VM_JNZ) && i.z == p + 2 && opof(c[p + 1]) == VM_RETK) {
            bool targeted = false;
            for (const auto& j : c)
                if (vm_is_jump(j) && j.z == p + 1) targeted = true;
            if (targeted) continue;
            i.op = op == VM_JZ ? VM_JNZRET : VM_JZRET;
            i.y = c[p + 1].y;
            i.z = 0;
            c[p + 1] = mxp_vm_ins{(uint8_t)VM_NOP, 0, 0, 0, 0, 0, 0};
        }
    }
    // 3. reachability
    std::vector<bool> reach(n, false);
    reach[0] = true;
    for (size_t p = 0; p < n; p++) {
        if (!reach[p]) continue;
        if (vm_is_jump(c[p])) reach[c[p].z] = true;
        if (!is_terminal(c[p]) && p + 1 < n) reach[p + 1] = true;
    }
    // 4. liveness (forward-only DAG: one backward sweep) and dead pure-op elimination
    std::vector<uint64_t> live_in(n + 1, 0);
    std::vector<bool> keep(n, true);
    for (size_t p = n; p-- > 0;) {
        if (!reach[p]) {
            keep[p] = false;
            live_in[p] = 0;
            continue;
        }
        const mxp_vm_ins& i = c[p];
        uint64_t out = 0;
        if (!is_terminal(i) && p + 1 < n) out |= live_in[p + 1];
        if (vm_is_jump(i)) out |= live_in[i.z];
        uint64_t w = writes(i);
        if (is_pure(i) && (w & out) == 0) {
            keep[p] = false;  // dead: forward to successor
            live_in[p] = out;
            if (opof(i) == VM_NOP || w == 0) live_in[p] = out;
            continue;
        }
        live_in[p] = reads(i) | (out & ~w);
    }
    // 5. a jump may target a removed instruction: retarget to the next kept one
    for (size_t p = 0; p < n; p++) {
        if (!keep[p] || !vm_is_jump(c[p])) continue;
        size_t t = c[p].z;
        while (t < n && !keep[t]) t++;
        if (t >= n) throw std::runtime_error("vmopt: jump past end");
        c[p].z = (uint32_t)t;
    }
    // 6. unconditional jumps over nothing but removed code are no-ops
    for (size_t p = 0; p < n; p++) {
        if (!keep[p] || opof(c[p]) != VM_JMP) continue;
        bool noop = true;
        for (size_t t = p + 1; t < c[p].z; t++)
            if (keep[t]) noop = false;
        if (noop) keep[p] = false;
    }
    relayout(c, keep);
}

void optimize_vm(std::vector<mxp_vm_ins>& c) {
    // a second round sees the layout of the first (e.g. JZ over a folded RETK becomes adjacent)
    optimize_once(c);
    optimize_once(c);
}

mxp_guard extract_guard(const std::vector<mxp_vm_ins>& c) {
    mxp_guard g{0, GM_NONE, 0, 0};
    if (c.size() < 3) return g;
    const mxp_vm_ins& a = c[0];
    const mxp_vm_ins& b = c[1];
    uint32_t kind;
    if (opof(a) == VM_RES && a.y <= W_D) kind = a.y;
    else if (opof(a) == VM_VCOL) kind = GK_VCOL;
    else return g;
    // `col.startsWith(K)`: a prefix atom (indexed by the leading bytes of the column value)
    const bool prefix = (kind == W_S || kind == GK_VCOL) && opof(b) == VM_STRFNK && b.y == SF_STARTS && b.a == 0 && b.d == 0 &&
                        !(b.op & MXP_VM_WAKE);
    if (a.d != 0 || (!prefix && (opof(b) != VM_EQK || b.a != 0 || b.d != 0 || (b.op & MXP_VM_WAKE)))) return g;
    size_t p = 2;
    uint32_t neg = 0;
    if (opof(c[p]) == VM_NOT && c[p].a == 0 && c[p].d == 0 && !(c[p].op & MXP_VM_WAKE)) {
        neg = 1;
        p++;
    }
    if (p >= c.size() || (c[p].op & MXP_VM_WAKE)) return g;
    const mxp_vm_ins& d = c[p];
    uint32_t mode;
    if (opof(d) == VM_JZRET && d.a == 0 && d.y == 0) mode = GM_AND;
    else if (opof(d) == VM_JNZRET && d.a == 0 && d.y == 1) mode = GM_OR;
    else if (opof(d) == VM_RET && d.a == 0 && d.y == 1) mode = GM_ONLY;
    else return g;
    // the continuation must not read register 0 (consumed by the decision)
    uint32_t cont = (uint32_t)(p + 1);
    if (mode != GM_ONLY) {
        if (cont >= c.size()) return g;
        // the decision popped r0: continuation code never reads it before writing (stack discipline)
    }
    g.col = a.x | (kind << 24);
    g.mode = mode | (neg << 8) | (cont << 16) | (prefix ? GT_PREFIX : 0u);
    g.klo = prefix ? b.x : b.y;
    g.khi = prefix ? 0u : b.z;
    return g;
}

bool hoist_continuation(const std::vector<mxp_vm_ins>& code, uint32_t pc0, HoistedCont* out) {
    out->code.assign(code.begin() + pc0, code.end());
    out->consts.clear();
    uint64_t used = 0;
    for (const auto& i : out->code) used |= reads(i) | writes(i);
    uint32_t next = 0;
    while (used >> next) next++;
    // the index kernels run templates in MXP_VM_MAXREG registers: a continuation that touches a
    // register past them (a deep rule, lower.cpp colouring onto MXP_VM_DEEPREG) is not templated, so
    // it never enters the index and keeps the deep kernels
    if (next > MXP_VM_MAXREG) return false;
    out->creg0 = next;
    for (auto& i : out->code) {
        const uint8_t wake = i.op & MXP_VM_WAKE;
        uint64_t k;
        switch (opof(i)) {
        case VM_EQK: k = (uint64_t)i.y | ((uint64_t)i.z << 32); i.op = VM_EQ; i.b = (uint8_t)next; i.y = i.z = 0; break;
        case VM_STRFNK: k = i.x; i.op = VM_STRFN; i.b = (uint8_t)next; i.x = 0; break;
        case VM_LOOKUPK: k = i.x; i.op = VM_LOOKUP; i.b = (uint8_t)next; i.x = 0; break;
        case VM_LOGICK: k = i.x; i.op = VM_LOGIC; i.b = (uint8_t)next; i.x = 0; break;
        case VM_CONST: k = (uint64_t)i.y | ((uint64_t)i.z << 32); i.op = VM_MOV; i.a = (uint8_t)next; i.y = i.z = 0; break;
        case VM_REGEX: k = i.x; i.op = VM_REGEXR; i.b = (uint8_t)next; i.x = 0; break;
        default: continue;
        }
        if (next >= MXP_VM_MAXREG) return false;
        i.op |= wake;
        out->consts.push_back(k);
        next++;
    }
    return true;
}

bool extract_second_prefix(const std::vector<mxp_vm_ins>& c, uint32_t pc0, SecondAtom* out) {
    if (pc0 + 3 > c.size()) return false;
    const mxp_vm_ins& r = c[pc0];
    const mxp_vm_ins& f = c[pc0 + 1];
    const mxp_vm_ins& d = c[pc0 + 2];
    if (((r.op | f.op | d.op) & MXP_VM_WAKE) || opof(r) != VM_RES || r.y != W_S) return false;
    if (opof(f) != VM_STRFNK || f.y != SF_STARTS || f.a != r.d) return false;
    out->col = r.x;
    out->k2 = f.x;
    if (opof(d) == VM_RET && d.a == f.d && d.y == 1) {
        out->direct = true;
        out->cont = pc0 + 3;
        return true;
    }
    if (opof(d) != VM_JZRET || d.a != f.d || d.y != 0) return false;
    const uint32_t cont = pc0 + 3;
    if (cont >= c.size()) return false;
    // forward dataflow over the continuation: registers that may still hold r / s (never rewritten
    // on some path from cont) must not be read
    std::vector<uint64_t> stale(c.size() + 1, 0);
    stale[cont] = (1ull << r.d) | (1ull << f.d);
    for (size_t pc = cont; pc < c.size(); pc++) {
        const mxp_vm_ins& i = c[pc];
        const uint64_t st = stale[pc];
        if (reads(i) & st) return false;
        const uint64_t w = writes(i);
        if (vm_is_jump(i)) {
            // TRES / try-LOOKUP write d only on the jump path
            if (i.z <= pc || i.z > c.size()) return false;
            stale[i.z] |= st & ~w;
            if (opof(i) != VM_JMP) stale[pc + 1] |= st;
        } else if (!is_terminal(i)) {
            stale[pc + 1] |= st & ~w;
        }
    }
    out->direct = false;
    out->cont = cont;
    return true;
}

}  // namespace mxp
