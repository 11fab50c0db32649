// wk_text.h -- host-side text formats shared by the weights files and the JSON config:
// .NET Core 3.0+ float formatting and a small JSON reader / writer (System.Text.Json
// defaults).  Host C++ only; nothing here touches a device.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace wk {

// float.ToString() (Number.Formatting FormatSingle, "G" shortest round trip).  en-US
// spells infinities "∞" (culture-dependent ToString in Matrix.Save); the invariant
// culture (System.Text.Json numbers) spells them "Infinity".
std::string dotnet_float(float v, bool invariant = false);

// A parsed JSON value (System.Text.Json document model reduced to what the config needs).
struct JsonValue {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  std::string text;  // Number: the raw token; String: the unescaped UTF-8 text
  std::vector<JsonValue> items;                              // Array
  std::vector<std::pair<std::string, JsonValue>> members;    // Object, in file order
};

// RFC 8259 JSON with System.Text.Json's default reader options: no comments, no trailing
// commas, depth <= 64, one root value.  Returns false with a message on error.
bool json_parse(const std::string& text, JsonValue& out, std::string& why);

// JavaScriptEncoder.Default string escaping (the serializer's default encoder): quotes,
// backslash, control characters, HTML-sensitive <>&'+` and all non-ASCII as \uXXXX.
std::string json_escape(const std::string& utf8);

// the thread's context-free error text (wk_last_error(NULL)); defined in wk_api.cpp
void set_last_error(const std::string& msg);

}  // namespace wk
