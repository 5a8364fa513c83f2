// ilgen.h -- Mixer IL (mixer/pkg/il) and its code generator (mixer/pkg/il/compiler).
//
// The engine compiles every rule to the *reference* IL first, with the reference's exact code
// generation (incl. its quirks), and only then lowers that IL to the GPU bytecode (lower.h).  This
// keeps the GPU path bit-exact by construction: whatever the reference's IL does, the lowering
// either reproduces or rejects.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "frontend.h"

namespace mxp {

// il.Type (mixer/pkg/il/types.go:23-48)
enum IlType : uint8_t { IL_UNKNOWN = 0, IL_VOID, IL_STRING, IL_INTEGER, IL_DOUBLE, IL_BOOL, IL_DURATION, IL_INTERFACE };
const char* il_type_name(uint8_t t);

// il.Opcode values (mixer/pkg/il/opcode.go:35-309)
enum Op : uint32_t {
    Halt = 0, Nop = 1, Err = 2, Errz = 3, Errnz = 4,
    PopS = 10, PopB = 11, PopI = 12, PopD = 13, DupS = 14, DupB = 15, DupI = 16, DupD = 17,
    RLoadS = 20, RLoadB = 21, RLoadI = 22, RLoadD = 23, ALoadS = 30, ALoadB = 31, ALoadI = 32, ALoadD = 33,
    APushS = 40, APushB = 41, APushI = 42, APushD = 43, RPushS = 50, RPushB = 51, RPushI = 52, RPushD = 53,
    EqS = 60, EqB = 61, EqI = 62, EqD = 63, AEqS = 70, AEqB = 71, AEqI = 72, AEqD = 73,
    Xor = 80, And = 81, Or = 82, AXor = 83, AAnd = 84, AOr = 85, Not = 86,
    ResolveS = 90, ResolveB = 91, ResolveI = 92, ResolveD = 93, ResolveF = 94,
    TResolveS = 100, TResolveB = 101, TResolveI = 102, TResolveD = 103, TResolveF = 104,
    AddI = 110, AddD = 111, SubI = 112, SubD = 113, AAddI = 114, AAddD = 115, ASubI = 116, ASubD = 117,
    Jmp = 200, Jz = 201, Jnz = 202, Call = 203, Ret = 204,
    Lookup = 210, TLookup = 211, ALookup = 212, NLookup = 213, ANLookup = 214
};

enum ArgKind : uint8_t { ARG_REG, ARG_STR, ARG_INT, ARG_DBL, ARG_BOOL, ARG_FN, ARG_ADDR };

struct OpInfo {
    const char* keyword;
    std::vector<ArgKind> args;
};
const OpInfo* op_info(uint32_t op);  // nullptr for unknown opcodes
uint32_t op_words(uint32_t op);

class StringTable {
  public:
    StringTable() { add("<<DEADBEEF>>"); }
    uint32_t add(const std::string& s);
    uint32_t try_id(const std::string& s) const;
    const std::string& get(uint32_t id) const { return strs_[id]; }
    size_t size() const { return strs_.size(); }

  private:
    std::unordered_map<std::string, uint32_t> ids_;
    std::vector<std::string> strs_;
};

struct IlFunction {
    uint32_t id = 0, address = 0, length = 0;
    std::vector<uint8_t> params;
    uint8_t ret = IL_VOID;
};

struct IlProgram {
    StringTable strings;
    std::map<uint32_t, IlFunction> functions;
    std::vector<uint32_t> code{Halt};
    bool add_function(const std::string& name, const std::vector<uint8_t>& params, uint8_t ret,
                      const std::vector<uint32_t>& body, std::string* err);
    const IlFunction* get(const std::string& name) const;
};

// Outcome of compiling one rule.
struct CompiledRule {
    enum Status { OK = 0, PARSE_ERROR = 1, TYPE_ERROR = 2, COMPILE_ERROR = 3, COMPILE_PANIC = 4 } status = OK;
    std::string error;        // the reference's error text for non-OK statuses
    int32_t value_type = 0;   // EvalType of the expression
    IlProgram program;        // "eval" function
};

// compiler.Compile (mixer/pkg/il/compiler/compiler.go:125-164)
void compile_rule(const std::string& text, const Vocabulary& vocab, const FuncMap& fmap, CompiledRule* out);

// text.WriteText (mixer/pkg/il/text/write.go:26-125)
std::string write_il_text(const IlProgram& p);

}  // namespace mxp
