// vmopt.h -- optimisation passes over lowered MXP VM programs and leading-atom guard extraction.
#pragma once

#include <vector>

#include "vm.h"

namespace mxp {

// Jump threading, constant-result folding (a jump whose target deterministically returns a
// constant bool becomes JZRET/JNZRET/RETK), dead pure-op elimination, unreachable-code removal and
// re-layout with WAKE flags.  Semantics-preserving for every lane; programs stay forward-only.
void optimize_vm(std::vector<mxp_vm_ins>& code);

// Guard of an optimised program (GM_NONE when the program does not start with a leading atom).
mxp_guard extract_guard(const std::vector<mxp_vm_ins>& code);

bool vm_is_jump(const mxp_vm_ins& i);

// Continuation template of a guarded rule: code[pc0, end) with every constant operand hoisted into
// a fresh register (EQK -> EQ, STRFNK -> STRFN, LOOKUPK -> LOOKUP, LOGICK -> LOGIC, CONST -> MOV),
// consts[j] being the value register creg0 + j must hold.  Jump targets keep their absolute pcs.
// Returns false when the continuation has no room for the extra registers.
struct HoistedCont {
    std::vector<mxp_vm_ins> code;
    std::vector<uint64_t> consts;
    uint32_t creg0 = 0;
};
bool hoist_continuation(const std::vector<mxp_vm_ins>& code, uint32_t pc0, HoistedCont* out);

// Second atom of an indexed `A == K1 && ...` rule: the continuation at pc0 starts with
//   RES col (want S) -> r ; STRFNK startsWith(r, K2) -> s ; JZRET s, false   (more code follows)
//                                                      or RET s (bool)      (the atom is the rest)
// and no later instruction can read r or s before rewriting them, so a lane whose column value
// starts with K2 may resume at `cont` with nothing else computed.  `direct`: the rule's result is
// the atom (a matching prefix is a true pair).
struct SecondAtom {
    uint32_t col = 0;
    uint32_t k2 = 0;    // prefix string id
    uint32_t cont = 0;  // resume pc (JZRET form)
    bool direct = false;
};
bool extract_second_prefix(const std::vector<mxp_vm_ins>& code, uint32_t pc0, SecondAtom* out);

}  // namespace mxp
