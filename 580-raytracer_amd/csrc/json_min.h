// json_min.h — a small JSON DOM reader for the scene format.
//
// Number semantics follow what the reference's loader does with nlohmann/json
// 3.11.3 (ExternalPlugins/json.hpp): a token without '.', 'e' or 'E' is an
// integer (strtoll/strtoull, json.hpp lexer), anything else goes through
// std::strtod (json.hpp:8290-8292); the scene code then narrows to float with
// static_cast (json.hpp:4694); a boolean converts to 1/0 like nlohmann's
// from_json for arithmetic types. Numbers follow the JSON grammar exactly as
// nlohmann's lexer does (no leading zeros, '+', leading or trailing '.'). A
// UTF-8 byte-order mark before the document is skipped. Objects keep the last
// value of a duplicated key and iterate in key order (nlohmann's std::map).
// Parse errors throw json_min::error, which the loaders turn into RT_FAILURE
// like the reference's try/catch (Raytracer.cpp:657-663, :775-778).
#pragma once
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace json_min {

struct error : std::runtime_error {
    explicit error(const std::string& m) : std::runtime_error(m) {}
};

struct Value {
    enum Kind { Null, Bool, Int, UInt, Float, String, Array, Object };
    Kind kind = Null;
    bool b = false;
    int64_t i = 0;
    uint64_t u = 0;
    double f = 0.0;
    std::string s;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;

    bool is_number() const { return kind == Int || kind == UInt || kind == Float; }
    bool is_array() const { return kind == Array; }
    bool is_object() const { return kind == Object; }
    bool is_string() const { return kind == String; }
    bool is_null() const { return kind == Null; }

    // json::get<float>() / implicit float conversion
    float as_float() const {
        switch (kind) {
            case Int: return static_cast<float>(i);
            case UInt: return static_cast<float>(u);
            case Float: return static_cast<float>(f);
            case Bool: return b ? 1.0f : 0.0f;
            default: throw error("type_error: number expected");
        }
    }
    int as_int() const {
        switch (kind) {
            case Int: return static_cast<int>(i);
            case UInt: return static_cast<int>(u);
            case Float: return static_cast<int>(f);
            case Bool: return b ? 1 : 0;
            default: throw error("type_error: number expected");
        }
    }
    const std::string& as_string() const {
        if (kind != String) throw error("type_error: string expected");
        return s;
    }
    bool contains(const std::string& k) const { return kind == Object && obj.count(k) != 0; }
    const Value& at(const std::string& k) const {
        if (kind != Object) throw error("type_error: object expected for key '" + k + "'");
        auto it = obj.find(k);
        if (it == obj.end()) throw error("out_of_range: key '" + k + "' not found");
        return it->second;
    }
    const Value& at(size_t idx) const {
        if (kind != Array) throw error("type_error: array expected");
        if (idx >= arr.size()) throw error("out_of_range: array index");
        return arr[idx];
    }
    size_t size() const { return kind == Array ? arr.size() : kind == Object ? obj.size() : 0; }
    // Elements in iteration order (array order, or object values in key order).
    std::vector<const Value*> items() const {
        std::vector<const Value*> out;
        if (kind == Array)
            for (auto& v : arr) out.push_back(&v);
        else if (kind == Object)
            for (auto& kv : obj) out.push_back(&kv.second);
        else if (kind != Null)
            out.push_back(this);
        return out;
    }
};

class Parser {
  public:
    explicit Parser(const std::string& text) : p_(text.c_str()), end_(text.c_str() + text.size()) {}
    Value parse_document() {
        if (end_ - p_ >= 3 && (unsigned char)p_[0] == 0xEF && (unsigned char)p_[1] == 0xBB &&
            (unsigned char)p_[2] == 0xBF)
            p_ += 3;  // UTF-8 BOM (nlohmann's lexer skips it)
        ws();
        Value v = value();
        ws();
        if (p_ != end_) fail("trailing characters");
        return v;
    }

  private:
    const char* p_;
    const char* end_;

    [[noreturn]] void fail(const char* m) { throw error(std::string("parse_error: ") + m); }
    void ws() {
        while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) p_++;
    }
    bool lit(const char* w) {
        size_t n = std::strlen(w);
        if ((size_t)(end_ - p_) >= n && std::memcmp(p_, w, n) == 0) { p_ += n; return true; }
        return false;
    }
    Value value() {
        if (p_ >= end_) fail("unexpected end");
        Value v;
        char c = *p_;
        if (c == '{') {
            v.kind = Value::Object;
            p_++;
            ws();
            if (p_ < end_ && *p_ == '}') { p_++; return v; }
            for (;;) {
                ws();
                if (p_ >= end_ || *p_ != '"') fail("object key expected");
                std::string k = str();
                ws();
                if (p_ >= end_ || *p_ != ':') fail("':' expected");
                p_++;
                ws();
                v.obj[k] = value();
                ws();
                if (p_ < end_ && *p_ == ',') { p_++; continue; }
                if (p_ < end_ && *p_ == '}') { p_++; break; }
                fail("',' or '}' expected");
            }
        } else if (c == '[') {
            v.kind = Value::Array;
            p_++;
            ws();
            if (p_ < end_ && *p_ == ']') { p_++; return v; }
            for (;;) {
                ws();
                v.arr.push_back(value());
                ws();
                if (p_ < end_ && *p_ == ',') { p_++; continue; }
                if (p_ < end_ && *p_ == ']') { p_++; break; }
                fail("',' or ']' expected");
            }
        } else if (c == '"') {
            v.kind = Value::String;
            v.s = str();
        } else if (lit("true")) {
            v.kind = Value::Bool; v.b = true;
        } else if (lit("false")) {
            v.kind = Value::Bool; v.b = false;
        } else if (lit("null")) {
            v.kind = Value::Null;
        } else if (c == '-' || (c >= '0' && c <= '9')) {
            number(v);
        } else {
            fail("unexpected character");
        }
        return v;
    }
    std::string str() {
        std::string out;
        p_++;  // opening quote
        while (p_ < end_ && *p_ != '"') {
            char c = *p_++;
            if ((unsigned char)c < 0x20) fail("control character in string");  // must be escaped (nlohmann)
            if (c == '\\') {
                if (p_ >= end_) fail("bad escape");
                char e = *p_++;
                switch (e) {
                    case '"': out += '"'; break;
                    case '\\': out += '\\'; break;
                    case '/': out += '/'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'n': out += '\n'; break;
                    case 'r': out += '\r'; break;
                    case 't': out += '\t'; break;
                    case 'u': {
                        if (end_ - p_ < 4) fail("bad \\u escape");
                        unsigned cp = (unsigned)std::strtoul(std::string(p_, 4).c_str(), nullptr, 16);
                        p_ += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: fail("bad escape");
                }
            } else {
                out += c;
            }
        }
        if (p_ >= end_) fail("unterminated string");
        p_++;
        return out;
    }
    bool digit() const { return p_ < end_ && *p_ >= '0' && *p_ <= '9'; }
    // -? (0 | [1-9][0-9]*) (. [0-9]+)? ([eE] [+-]? [0-9]+)?  (RFC 8259; what
    // nlohmann's lexer accepts; a digit right after a leading 0 ends the
    // number there and the parser then rejects the next token)
    void number(Value& v) {
        const char* s = p_;
        if (*p_ == '-') p_++;
        if (!digit()) fail("bad number");
        if (*p_ == '0') p_++;
        else
            while (digit()) p_++;
        bool is_float = false;
        if (p_ < end_ && *p_ == '.') {
            is_float = true;
            p_++;
            if (!digit()) fail("bad number: digit expected after '.'");
            while (digit()) p_++;
        }
        if (p_ < end_ && (*p_ == 'e' || *p_ == 'E')) {
            is_float = true;
            p_++;
            if (p_ < end_ && (*p_ == '+' || *p_ == '-')) p_++;
            if (!digit()) fail("bad number: digit expected in exponent");
            while (digit()) p_++;
        }
        std::string tok(s, p_);
        char* e = nullptr;
        if (!is_float) {
            errno = 0;
            if (tok[0] == '-') {
                long long x = std::strtoll(tok.c_str(), &e, 10);
                if (errno == 0 && e && *e == 0) { v.kind = Value::Int; v.i = x; return; }
            } else {
                unsigned long long x = std::strtoull(tok.c_str(), &e, 10);
                if (errno == 0 && e && *e == 0) {
                    if (x <= (unsigned long long)INT64_MAX) { v.kind = Value::Int; v.i = (int64_t)x; }
                    else { v.kind = Value::UInt; v.u = x; }
                    return;
                }
            }
            // out of 64-bit range: nlohmann falls back to a floating-point value
        }
        v.kind = Value::Float;
        v.f = std::strtod(tok.c_str(), &e);
        if (!e || *e != 0) fail("bad number");
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse_document(); }

}  // namespace json_min
