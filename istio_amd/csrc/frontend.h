// frontend.h -- Mixer expression language front end (host side of the engine).
//
// Parses the Go-expression subset accepted by `expr.Parse` (mixer/pkg/expr/expr.go:424-436, which
// delegates to go/parser.ParseExpr), converts it to Mixer's expression tree (`process`,
// expr.go:287-421) and type checks it against the attribute vocabulary (`EvalType`,
// expr.go:93-105, 202-268) using the intrinsic table of mixer/pkg/expr/func.go:39-72 and the extern
// metadata of mixer/pkg/il/runtime/externs.go:42-79.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace mxp {

// istio.io/api mixer/v1/config/descriptor ValueType
enum ValueType : int32_t {
    VT_UNSPECIFIED = 0, VT_STRING = 1, VT_INT64 = 2, VT_DOUBLE = 3, VT_BOOL = 4, VT_TIMESTAMP = 5,
    VT_IP_ADDRESS = 6, VT_EMAIL_ADDRESS = 7, VT_URI = 8, VT_DNS_NAME = 9, VT_DURATION = 10,
    VT_STRING_MAP = 11
};
const char* value_type_name(int32_t vt);

struct Expr;
using ExprP = std::unique_ptr<Expr>;

struct Constant {
    std::string src;    // literal text as written (Constant.String)
    int32_t type = 0;   // ValueType
    // typed value
    std::string s;      // STRING
    int64_t i = 0;      // INT64, DURATION
    double d = 0;       // DOUBLE
    bool b = false;     // BOOL
};

struct Expr {
    enum Kind { EMPTY, CONST, VAR, FN } kind = EMPTY;
    Constant c;
    std::string var;            // attribute name
    std::string fn;             // function name
    ExprP target;               // instance-method receiver
    std::vector<ExprP> args;
    std::string str() const;    // postfix form (Expression.String)
};

struct FunctionMetadata {
    std::string name;
    bool instance = false;
    int32_t target_type = VT_UNSPECIFIED;
    int32_t return_type = VT_UNSPECIFIED;
    std::vector<int32_t> arg_types;
};

using Vocabulary = std::map<std::string, int32_t>;           // attribute name -> ValueType
using FuncMap = std::map<std::string, FunctionMetadata>;

FuncMap default_func_map();

enum class FrontError { NONE, PARSE, TYPE, PANIC };

// expr.Parse: on failure returns nullptr and the reference's error text.
ExprP parse_expression(const std::string& src, std::string* err);
// Expression.EvalType: returns false with the error text (or a panic marker).
bool eval_type(const Expr& e, const Vocabulary& v, const FuncMap& f, int32_t* out, std::string* err,
               bool* panicked);

}  // namespace mxp
