// qkd_json.hpp — the small JSON reader the batch driver needs for the
// reference's config.json (src/config.cpp reads it with nlohmann::json, a
// dependency this build does not carry). Objects, arrays, numbers, strings,
// booleans and null; numbers are kept as text and converted on access, as
// `get<size_t>()` / `get<double>()` would. Errors throw std::runtime_error.
#pragma once
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace qkdjson {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    std::string text;                                   // number literal or string
    std::vector<Value> items;                           // array
    std::vector<std::pair<std::string, Value>> fields;  // object, in file order

    const Value& operator[](const std::string& key) const {
        if (kind != Object) throw std::runtime_error("[json.exception.type_error] cannot use operator[] with a string argument on a non-object");
        for (const auto& f : fields)
            if (f.first == key) return f.second;
        throw std::runtime_error("[json.exception.type_error] key '" + key + "' not found");
    }
    bool contains(const std::string& key) const {
        if (kind != Object) return false;
        for (const auto& f : fields)
            if (f.first == key) return true;
        return false;
    }
    bool as_bool() const {
        if (kind != Bool) throw std::runtime_error("[json.exception.type_error] type must be boolean");
        return b;
    }
    double as_double() const {
        if (kind != Number) throw std::runtime_error("[json.exception.type_error] type must be number");
        return std::strtod(text.c_str(), nullptr);
    }
    // get<size_t>(): non-negative integers (a fractional value truncates, a
    // negative one is rejected rather than wrapped)
    size_t as_size() const {
        if (kind != Number) throw std::runtime_error("[json.exception.type_error] type must be number");
        if (!text.empty() && text[0] == '-') throw std::runtime_error("[json.exception.type_error] value must be non-negative");
        if (text.find_first_of(".eE") != std::string::npos) return (size_t)std::strtod(text.c_str(), nullptr);
        errno = 0;
        const unsigned long long v = std::strtoull(text.c_str(), nullptr, 10);
        if (errno == ERANGE) throw std::runtime_error("[json.exception.out_of_range] integer out of range");
        return (size_t)v;
    }
};

class Parser {
  public:
    explicit Parser(const std::string& s) : s_(s) {}
    Value parse() {
        Value v = value();
        ws();
        if (p_ != s_.size()) error("unexpected trailing characters");
        return v;
    }

  private:
    const std::string& s_;
    size_t p_ = 0;

    [[noreturn]] void error(const std::string& what) const {
        throw std::runtime_error("[json.exception.parse_error] at byte " + std::to_string(p_ + 1) + ": " + what);
    }
    void ws() {
        while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
    }
    bool eat(char c) {
        ws();
        if (p_ < s_.size() && s_[p_] == c) {
            ++p_;
            return true;
        }
        return false;
    }
    void expect(char c) {
        if (!eat(c)) error(std::string("expected '") + c + "'");
    }
    Value value() {
        ws();
        if (p_ >= s_.size()) error("unexpected end of input");
        const char c = s_[p_];
        Value v;
        if (c == '{') {
            ++p_;
            v.kind = Value::Object;
            if (eat('}')) return v;
            do {
                ws();
                std::string k = str();
                expect(':');
                v.fields.emplace_back(std::move(k), value());
            } while (eat(','));
            expect('}');
        } else if (c == '[') {
            ++p_;
            v.kind = Value::Array;
            if (eat(']')) return v;
            do v.items.push_back(value());
            while (eat(','));
            expect(']');
        } else if (c == '"') {
            v.kind = Value::String;
            v.text = str();
        } else if (s_.compare(p_, 4, "true") == 0) {
            p_ += 4;
            v.kind = Value::Bool;
            v.b = true;
        } else if (s_.compare(p_, 5, "false") == 0) {
            p_ += 5;
            v.kind = Value::Bool;
        } else if (s_.compare(p_, 4, "null") == 0) {
            p_ += 4;
        } else if (c == '-' || std::isdigit((unsigned char)c)) {
            const size_t b = p_;
            if (s_[p_] == '-') ++p_;
            while (p_ < s_.size() && (std::isdigit((unsigned char)s_[p_]) || s_[p_] == '.' || s_[p_] == 'e' ||
                                      s_[p_] == 'E' || s_[p_] == '+' || s_[p_] == '-'))
                ++p_;
            v.kind = Value::Number;
            v.text = s_.substr(b, p_ - b);
            char* end = nullptr;
            std::strtod(v.text.c_str(), &end);
            if (v.text.empty() || end != v.text.c_str() + v.text.size()) error("invalid number '" + v.text + "'");
        } else {
            error(std::string("unexpected character '") + c + "'");
        }
        return v;
    }
    std::string str() {
        if (p_ >= s_.size() || s_[p_] != '"') error("expected string");
        ++p_;
        std::string out;
        while (p_ < s_.size() && s_[p_] != '"') {
            char c = s_[p_++];
            if (c == '\\') {
                if (p_ >= s_.size()) error("unterminated escape");
                const char e = s_[p_++];
                switch (e) {
                    case 'n': c = '\n'; break;
                    case 't': c = '\t'; break;
                    case 'r': c = '\r'; break;
                    case 'b': c = '\b'; break;
                    case 'f': c = '\f'; break;
                    case 'u': {
                        if (p_ + 4 > s_.size()) error("bad \\u escape");
                        const unsigned cp = (unsigned)std::strtoul(s_.substr(p_, 4).c_str(), nullptr, 16);
                        p_ += 4;
                        if (cp < 0x80) {
                            out += (char)cp;
                        } else if (cp < 0x800) {
                            out += (char)(0xC0 | (cp >> 6));
                            out += (char)(0x80 | (cp & 0x3F));
                        } else {
                            out += (char)(0xE0 | (cp >> 12));
                            out += (char)(0x80 | ((cp >> 6) & 0x3F));
                            out += (char)(0x80 | (cp & 0x3F));
                        }
                        continue;
                    }
                    default: c = e;
                }
            }
            out += c;
        }
        if (p_ >= s_.size()) error("unterminated string");
        ++p_;
        return out;
    }
};

inline Value parse(const std::string& text) {
    // a UTF-8 byte-order mark (the reference's own sources carry one) is skipped
    const size_t skip = text.compare(0, 3, "\xEF\xBB\xBF") == 0 ? 3 : 0;
    const std::string body = text.substr(skip);
    return Parser(body).parse();
}

}  // namespace qkdjson
