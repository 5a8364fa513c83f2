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

}  // namespace mxp
