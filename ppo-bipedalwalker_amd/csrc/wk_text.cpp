// wk_text.cpp -- see wk_text.h.
#include "wk_text.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace wk {

std::string dotnet_float(float v, bool invariant) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) {
    if (invariant) return v > 0 ? "Infinity" : "-Infinity";
    return v > 0 ? "\xe2\x88\x9e" : "-\xe2\x88\x9e";
  }
  if (v == 0.0f) return std::signbit(v) ? "-0" : "0";
  // shortest round-trip digits: the fewest significant digits p for which some p-digit
  // decimal reads back as v, choosing the one nearest v.  The correctly rounded p-digit
  // value is the nearest; at a power of two the round-trip interval is asymmetric, so its
  // neighbour one unit in the last place up may round-trip when the nearest does not.
  char buf[64];
  std::string digits;
  int exp10 = 0;
  bool neg = v < 0;
  for (int prec = 1; prec <= 9; prec++) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, (double)std::fabs(v));
    const char* e = strchr(buf, 'e');
    std::string d;
    for (const char* q = buf; q < e; q++)
      if (*q != '.') d += *q;
    const int x = atoi(e + 1);
    bool ok = strtof(buf, nullptr) == std::fabs(v);
    if (!ok) {  // try the next p-digit decimal above and below
      for (int dir = -1; dir <= 1 && !ok; dir += 2) {
        long long m = atoll(d.c_str()) + dir;
        long long lo = 1;
        for (int i = 1; i < prec; i++) lo *= 10;
        int xx = x;
        if (m < lo) { m = lo * 10 - 1; xx--; }      // 1000 - 1 -> 9999 one decade down
        if (m >= lo * 10) { m = lo; xx++; }          // 9999 + 1 -> 1000 one decade up
        char cand[64];
        snprintf(cand, sizeof cand, "%llde%d", m, xx - (prec - 1));
        if (strtof(cand, nullptr) == std::fabs(v)) {
          ok = true;
          d = std::to_string(m);
          exp10 = xx;
        }
      }
      if (!ok) continue;
    } else {
      exp10 = x;
    }
    digits = d;
    break;
  }
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out = neg ? "-" : "";
  // Number.Formatting FormatGeneral: scientific when the decimal-point position
  // (exp10 + 1) exceeds max(digit count, SinglePrecision = 9) or is below -3
  const int scale = exp10 + 1;
  if (scale > std::max((int)digits.size(), 9) || scale < -3) {  // d[.ddd]E+XX
    out += digits[0];
    if (digits.size() > 1) out += "." + digits.substr(1);
    char eb[16];
    snprintf(eb, sizeof eb, "E%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
    out += eb;
  } else if (exp10 < 0) {
    out += "0." + std::string(-exp10 - 1, '0') + digits;
  } else if ((int)digits.size() <= exp10 + 1) {
    out += digits + std::string(exp10 + 1 - digits.size(), '0');
  } else {
    out += digits.substr(0, exp10 + 1) + "." + digits.substr(exp10 + 1);
  }
  return out;
}

namespace {
struct Reader {
  const std::string& s;
  size_t i = 0;
  std::string why;
  explicit Reader(const std::string& t) : s(t) {}
  bool fail(const char* m) {
    char b[160];
    snprintf(b, sizeof b, "%s at byte %zu", m, i);
    why = b;
    return false;
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 63)); }
    else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63));
    } else {
      o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 63));
      o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63));
    }
  }
  bool hex4(uint32_t& v) {
    if (i + 4 > s.size()) return fail("truncated \\u escape");
    v = 0;
    for (int k = 0; k < 4; k++) {
      const char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else return fail("bad \\u escape");
    }
    return true;
  }
  bool string(std::string& o) {
    i++;  // opening quote
    while (true) {
      if (i >= s.size()) return fail("unterminated string");
      const unsigned char c = (unsigned char)s[i];
      if (c == '"') { i++; return true; }
      if (c < 0x20) return fail("control character in string");
      if (c != '\\') { o += (char)c; i++; continue; }
      if (++i >= s.size()) return fail("unterminated escape");
      const char e = s[i++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {  // surrogate pair
            uint32_t lo;
            if (i + 2 > s.size() || s[i] != '\\' || s[i + 1] != 'u') return fail("lone surrogate");
            i += 2;
            if (!hex4(lo)) return false;
            if (lo < 0xDC00 || lo >= 0xE000) return fail("bad surrogate pair");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp < 0xE000) {
            return fail("lone surrogate");
          }
          put_utf8(o, cp);
          break;
        }
        default: return fail("bad escape");
      }
    }
  }
  bool number(std::string& o) {
    const size_t a = i;
    if (s[i] == '-') i++;
    if (i >= s.size()) return fail("bad number");
    if (s[i] == '0') i++;
    else if (s[i] >= '1' && s[i] <= '9') while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    else return fail("bad number");
    if (i < s.size() && s[i] == '.') {
      i++;
      if (i >= s.size() || !isdigit((unsigned char)s[i])) return fail("bad number");
      while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
      i++;
      if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
      if (i >= s.size() || !isdigit((unsigned char)s[i])) return fail("bad number");
      while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    }
    o = s.substr(a, i - a);
    return true;
  }
  bool lit(const char* w) {
    const size_t n = strlen(w);
    if (s.compare(i, n, w) != 0) return fail("invalid literal");
    i += n;
    return true;
  }
  bool value(JsonValue& v, int depth) {
    if (depth > 64) return fail("maximum depth 64 exceeded");
    ws();
    if (i >= s.size()) return fail("unexpected end of data");
    const char c = s[i];
    if (c == '{') {
      v.kind = JsonValue::Object;
      i++;
      ws();
      if (i < s.size() && s[i] == '}') { i++; return true; }
      while (true) {
        ws();
        if (i >= s.size() || s[i] != '"') return fail("expected property name");
        std::string name;
        if (!string(name)) return false;
        ws();
        if (i >= s.size() || s[i] != ':') return fail("expected ':'");
        i++;
        JsonValue m;
        if (!value(m, depth + 1)) return false;
        v.members.emplace_back(std::move(name), std::move(m));
        ws();
        if (i < s.size() && s[i] == ',') { i++; continue; }
        if (i < s.size() && s[i] == '}') { i++; return true; }
        return fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      v.kind = JsonValue::Array;
      i++;
      ws();
      if (i < s.size() && s[i] == ']') { i++; return true; }
      while (true) {
        JsonValue m;
        if (!value(m, depth + 1)) return false;
        v.items.push_back(std::move(m));
        ws();
        if (i < s.size() && s[i] == ',') { i++; continue; }
        if (i < s.size() && s[i] == ']') { i++; return true; }
        return fail("expected ',' or ']'");
      }
    }
    if (c == '"') { v.kind = JsonValue::String; return string(v.text); }
    if (c == 't') { v.kind = JsonValue::Bool; v.b = true; return lit("true"); }
    if (c == 'f') { v.kind = JsonValue::Bool; v.b = false; return lit("false"); }
    if (c == 'n') { v.kind = JsonValue::Null; return lit("null"); }
    v.kind = JsonValue::Number;
    return number(v.text);
  }
};
}  // namespace

bool json_parse(const std::string& text, JsonValue& out, std::string& why) {
  Reader r(text);
  // a UTF-8 byte order mark is skipped (File.OpenRead + JsonSerializer.Deserialize)
  if (text.compare(0, 3, "\xEF\xBB\xBF") == 0) r.i = 3;
  if (!r.value(out, 0)) { why = r.why; return false; }
  r.ws();
  if (r.i != text.size()) { r.fail("data after the root value"); why = r.why; return false; }
  return true;
}

std::string json_escape(const std::string& u) {
  std::string o;
  char b[16];
  for (size_t i = 0; i < u.size();) {
    const unsigned char c = (unsigned char)u[i];
    uint32_t cp;
    int len;
    if (c < 0x80) { cp = c; len = 1; }
    else if ((c >> 5) == 6 && i + 1 < u.size()) { cp = ((c & 31u) << 6) | (u[i + 1] & 63u); len = 2; }
    else if ((c >> 4) == 14 && i + 2 < u.size()) {
      cp = ((c & 15u) << 12) | ((u[i + 1] & 63u) << 6) | (u[i + 2] & 63u); len = 3;
    } else if ((c >> 3) == 30 && i + 3 < u.size()) {
      cp = ((c & 7u) << 18) | ((u[i + 1] & 63u) << 12) | ((u[i + 2] & 63u) << 6) | (u[i + 3] & 63u);
      len = 4;
    } else { cp = 0xFFFD; len = 1; }
    i += len;
    switch (cp) {
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\\': o += "\\\\"; continue;
      default: break;
    }
    const bool plain = cp >= 0x20 && cp < 0x7F && !strchr("\"<>&'+`", (int)cp);
    if (plain) { o += (char)cp; continue; }
    if (cp >= 0x10000) {  // UTF-16 surrogate pair
      const uint32_t v = cp - 0x10000;
      snprintf(b, sizeof b, "\\u%04X\\u%04X", 0xD800 + (v >> 10), 0xDC00 + (v & 0x3FF));
    } else {
      snprintf(b, sizeof b, "\\u%04X", cp);
    }
    o += b;
  }
  return o;
}

}  // namespace wk
