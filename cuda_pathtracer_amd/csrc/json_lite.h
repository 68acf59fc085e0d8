// Minimal JSON reader for scene files (replaces the vendored nlohmann::json 3.11.3 used by
// path_tracer/src/scene.cpp:33-219).  Semantics the scene format depends on:
//   * objects iterate in SORTED key order — nlohmann::json's default object type is std::map,
//     so the reference assigns material ids alphabetically (scene.cpp:42-57);
//   * a duplicate key keeps the last value (std::map assignment during parse);
//   * numbers are parsed as double (strtod, correctly rounded) and narrowed to float by the
//     caller, as `p.value("RGB", std::vector<float>)` does.
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace jl {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;

    bool has(const std::string& k) const { return kind == Object && obj.count(k) != 0; }
    const Value& operator[](const std::string& k) const {
        auto it = obj.find(k);
        if (kind != Object || it == obj.end()) throw std::runtime_error("missing key '" + k + "'");
        return it->second;
    }
    const Value& operator[](size_t i) const {
        if (kind != Array || i >= arr.size()) throw std::runtime_error("array index out of range");
        return arr[i];
    }
    double number() const {
        if (kind != Number) throw std::runtime_error("expected a number");
        return num;
    }
    const std::string& string() const {
        if (kind != String) throw std::runtime_error("expected a string");
        return str;
    }
};

class Parser {
public:
    explicit Parser(const std::string& s) : s_(s) {}
    Value parse() {
        Value v = value();
        ws();
        if (i_ != s_.size()) err("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t i_ = 0;

    [[noreturn]] void err(const char* m) { throw std::runtime_error(std::string("json: ") + m + " at offset " + std::to_string(i_)); }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
    }
    bool lit(const char* w) {
        size_t n = std::char_traits<char>::length(w);
        if (s_.compare(i_, n, w) == 0) { i_ += n; return true; }
        return false;
    }
    Value value() {
        ws();
        if (i_ >= s_.size()) err("unexpected end");
        const char c = s_[i_];
        Value v;
        if (c == '{') {
            v.kind = Value::Object;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
            for (;;) {
                ws();
                if (i_ >= s_.size() || s_[i_] != '"') err("expected key");
                std::string k = string_body();
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') err("expected ':'");
                ++i_;
                v.obj[k] = value();
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
                if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
                err("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = Value::Array;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
                if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
                err("expected ',' or ']'");
            }
        }
        if (c == '"') { v.kind = Value::String; v.str = string_body(); return v; }
        if (lit("true")) { v.kind = Value::Bool; v.b = true; return v; }
        if (lit("false")) { v.kind = Value::Bool; v.b = false; return v; }
        if (lit("null")) return v;
        if (c == '-' || (c >= '0' && c <= '9')) {
            const char* b = s_.c_str() + i_;
            char* e = nullptr;
            v.kind = Value::Number;
            v.num = std::strtod(b, &e);
            if (e == b) err("bad number");
            i_ += (size_t)(e - b);
            return v;
        }
        err("unexpected character");
    }
    std::string string_body() {
        ++i_;  // opening quote
        std::string out;
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\') {
                if (i_ >= s_.size()) err("bad escape");
                char e = s_[i_++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (i_ + 4 > s_.size()) err("bad \\u escape");
                        unsigned cp = (unsigned)std::stoul(s_.substr(i_, 4), nullptr, 16);
                        i_ += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += e; break;
                }
            } else {
                out += c;
            }
        }
        if (i_ >= s_.size()) err("unterminated string");
        ++i_;
        return out;
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace jl
