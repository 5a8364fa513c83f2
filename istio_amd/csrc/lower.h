// lower.h -- reference IL -> MXP VM bytecode (vm.h).
//
// The lowering abstract-interprets the IL of `compile_rule` over a typed value stack, one copy of
// the code per (IL address, stack shape), so every stack slot maps to one fixed register and all
// jumps go forward.  The reference's stack (64 words) and heap (64 slots) limits are reproduced
// where a path can reach them ("stack overflow", "heap overflow", Go's index panic; lower.cpp).
// A program the lowering cannot express (more than MXP_VM_MAXREG values live at once, more than
// kMaxContexts shape contexts) is reported (LoweredRule::ok == false), not approximated.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "ilgen.h"
#include "vm.h"

namespace mxp {

// Engine-global tables the lowering interns constants and columns into.
enum RxSource { RX_SRC_COLUMN = 0, RX_SRC_VCOLUMN = 1, RX_SRC_MAPVALS = 2, RX_SRC_CONST = 3 };

class LowerTables {
  public:
    virtual ~LowerTables() = default;
    virtual uint32_t intern_string(const std::string& s) = 0;     // global string id
    // []byte value -> packed id: canonical-form id (net.IP.Equal classes) << 28 | raw-bytes id
    virtual uint64_t intern_bytes(const std::string& raw) = 0;
    virtual uint32_t intern_time(int64_t sec, int32_t nsec) = 0;  // time id
    virtual uint32_t column(const std::string& attr) = 0;         // resolve column index
    virtual uint32_t vcolumn(const std::string& attr, const std::string& key) = 0;  // map[key] column
    virtual int32_t attr_type(const std::string& attr) = 0;       // manifest ValueType (-1 unknown)
    // constant regexp pattern -> rule-set DFA index; -1 syntax error, -2 unsupported (err says why)
    virtual int32_t regex_const(const std::string& pattern, std::string* err) = 0;
    virtual bool regex_const_match(int32_t dfa, const std::string& subject) = 0;
    // values used as run-time regexp patterns (the packer compiles each distinct one per batch):
    // an attribute's string values, a map attribute's [key] values or all its values, a constant
    virtual void regex_source(int kind, const std::string& attr, const std::string& key, uint32_t sid) = 0;
};

struct LoweredRule {
    bool ok = false;
    std::string why;              // reason when !ok
    std::vector<mxp_vm_ins> code;
    uint32_t nregs = 0;
    bool uses_ipof = false;
    bool uses_tsof = false;
    bool uses_strings = false;    // needs string bytes on device (dynamic string functions)
    bool uses_maps = false;       // needs per-request map storage on device
    bool uses_rxof = false;       // run-time regexp patterns (per-batch pattern DFAs)
};

LoweredRule lower_rule(const IlProgram& prog, LowerTables* tables);

std::string vm_disasm(const std::vector<mxp_vm_ins>& code);

}  // namespace mxp
