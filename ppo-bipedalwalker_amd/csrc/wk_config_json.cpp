// wk_config_json.cpp -- the reference's JSON configuration files.
//
// Hyperparameters.SerializeJson / DeserializeJson (Hyperparameters.cs:124-187) move a
// SerializableHyperparameters object (Hyperparameters.cs:11-77) through System.Text.Json
// with default options (WriteIndented on save).  Here the same document maps onto
// wk_config (the kernels' hyperparameters) plus wk_host_settings (the host-only fields:
// CollectData, SaveWeights, file names, FilePath, and the network DSL strings' storage).
//
// Load semantics follow the reference step by step:
//   1. deserialize: unknown properties are ignored, a missing property keeps the current
//      value (the serializable object's constructor copies the current settings), the last
//      duplicate wins, property names are case-sensitive; a type mismatch, a non-finite or
//      out-of-range number, comments or trailing commas fail ("JSON deserializer error");
//   2. ValidateHyperparameterValues (:189-217) on the result -- any violation fails and
//      nothing is applied;
//   3. apply, then ValidateVariables (:240-290): an invalid FilePath, weights file name or
//      network DSL string is reset to its default and reported.  The return value counts
//      those corrections (0 = none); their messages, one per line, are in wk_last_error(NULL).
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <regex>
#include <string>

#include "../../include/wk_api.h"
#include "wk_text.h"

namespace {

const char* kCriticDefault = "Input |64| (LeakyReLU) |1| Output";
const char* kActorDefault = "Input |64| (LeakyReLU) |64| (LeakyReLU) |4| (TanH) Output";

// AppDomain.CurrentDomain.BaseDirectory: the running executable's directory, with "/"
std::string base_directory() {
  char b[4096];
  const ssize_t n = readlink("/proc/self/exe", b, sizeof b - 1);
  if (n <= 0) return "./";
  std::string p(b, (size_t)n);
  return p.substr(0, p.rfind('/') + 1);
}

void copy_str(char* dst, size_t cap, const std::string& s) {
  const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
  memcpy(dst, s.data(), n);
  dst[n] = 0;
}

// ConsoleRenderer.ValidateFileName (ConsoleRenderer.cs:639-647): Path.GetInvalidFileNameChars
// on Linux is { '\0', '/' }
bool valid_file_name(const char* s) { return s && !strchr(s, '/'); }

// ConsoleRenderer.ValidateFilePath (:650-658)
bool valid_file_path(const char* s) {
  if (!s || !*s) return false;
  const size_t n = strlen(s);
  struct stat st;
  return s[n - 1] == '/' && stat(s, &st) == 0 && S_ISDIR(st.st_mode);
}

// ConsoleRenderer.ValidateNeuralNetwork (:661-682)
bool valid_network(const char* s, bool critic, std::string& why) {
  if (!s) { why = "neural network not valid, check syntax"; return false; }
  static const std::regex pat("^Input ((\\|[1-9][0-9]*\\| )|(\\((LeakyReLU|TanH|ReLU)\\) ))+Output$");
  if (!std::regex_match(s, pat)) { why = "neural network not valid, check syntax"; return false; }
  const std::string t(s);
  const size_t b = t.rfind('|'), a = t.rfind('|', b - 1);
  const long out = strtol(t.substr(a + 1, b - a - 1).c_str(), nullptr, 10);
  const long need = critic ? 1 : 4;
  if (out != need) {
    why = "last dense layer should output " + std::to_string(need) + ", currently outputs " +
          std::to_string(out);
    return false;
  }
  return true;
}

// System.Text.Json number conversions (Utf8JsonReader.TryGetInt32 / TryGetSingle)
bool get_int(const wk::JsonValue& v, int& out) {
  if (v.kind != wk::JsonValue::Number) return false;
  const std::string& t = v.text;
  if (t.find_first_of(".eE") != std::string::npos) return false;
  errno = 0;
  char* end = nullptr;
  const long long x = strtoll(t.c_str(), &end, 10);
  if (*end || errno || x < INT32_MIN || x > INT32_MAX) return false;
  out = (int)x;
  return true;
}
bool get_float(const wk::JsonValue& v, float& out) {
  if (v.kind != wk::JsonValue::Number) return false;
  char* end = nullptr;
  const float x = strtof(v.text.c_str(), &end);
  if (*end || !std::isfinite(x)) return false;
  out = x;
  return true;
}

struct Fields {  // SerializableHyperparameters, in declaration (= serialization) order
  int GameSpeed, CollectData, SaveWeights, Iterations, MaxTimesteps, RoughFloor;
  std::string CriticNeuralNetwork, ActorNeuralNetwork, CriticWeightFileName, ActorWeightFileName,
      FilePath;
  bool critic_null, actor_null, cname_null, aname_null, path_null;
  float Alpha, Beta1, Beta2, AdamEpsilon;
  int Epochs, BatchSize, UseGAE, NormalizeAdvantages;
  float Gamma, Lambda, Epsilon, LogStandardDeviation;
};

Fields from(const wk_config* c, const wk_host_settings* h) {
  Fields f{};
  f.GameSpeed = c->GameSpeed; f.CollectData = h->CollectData; f.SaveWeights = h->SaveWeights;
  f.Iterations = c->Iterations; f.MaxTimesteps = c->MaxTimesteps; f.RoughFloor = c->RoughFloor != 0;
  f.CriticNeuralNetwork = c->CriticNeuralNetwork ? c->CriticNeuralNetwork : kCriticDefault;
  f.ActorNeuralNetwork = c->ActorNeuralNetwork ? c->ActorNeuralNetwork : kActorDefault;
  f.CriticWeightFileName = h->CriticWeightFileName; f.ActorWeightFileName = h->ActorWeightFileName;
  f.FilePath = h->FilePath;
  f.Alpha = c->Alpha; f.Beta1 = c->Beta1; f.Beta2 = c->Beta2; f.AdamEpsilon = c->AdamEpsilon;
  f.Epochs = c->Epochs; f.BatchSize = c->BatchSize; f.UseGAE = c->UseGAE != 0;
  f.NormalizeAdvantages = c->NormalizeAdvantages != 0;
  f.Gamma = c->Gamma; f.Lambda = c->Lambda; f.Epsilon = c->Epsilon;
  f.LogStandardDeviation = c->LogStandardDeviation;
  return f;
}

// ValidateHyperparameterValues (Hyperparameters.cs:189-217), the reference's messages
std::string validate_values(const Fields& h) {
  char b[160];
  auto num = [&](const char* m, double v) { snprintf(b, sizeof b, m, v); return std::string(b); };
  if (h.GameSpeed <= 0 || h.GameSpeed >= 10) return num("Invalid game speed, should be in range 0<x<10 (%g)", h.GameSpeed);
  if (h.Iterations <= 0 || h.Iterations >= 200) return num("Invalid iterations count, should be in range 0<x<200 (%g)", h.Iterations);
  if (h.MaxTimesteps <= 0) return num("Invalid maximum time steps amount, should be in range x>0 (%g)", h.MaxTimesteps);
  if (h.Alpha <= 0 || h.Alpha >= 10) return num("Invalid alpha value, should be in range 0<x<10 (%g)", h.Alpha);
  if (h.Beta1 <= 0 || h.Beta1 > 1) return num("Invalid beta1 value, should be in range 0<x<1 (%g", h.Beta1);
  if (h.Beta2 <= 0 || h.Beta2 > 1) return num("Invalid beta2 value, should be in range 0<x<1 (%g)", h.Beta2);
  if (h.AdamEpsilon <= 0 || h.AdamEpsilon >= 1) return num("Invalid Adam epsilon value, should be in range 0<x<1 (%g)", h.AdamEpsilon);
  if (h.Epochs <= 0 || h.Epochs >= 50) return num("Invalid epochs value, should be in range 0<x<50 (%g)", h.Epochs);
  if (h.BatchSize <= 0 || h.BatchSize >= 1000) return num("Invalid batch size value, should be in range 0<x<1000 (%g)", h.BatchSize);
  if (h.Gamma <= 0 || h.Gamma > 1) return num("Invalid gamma value, should be in range 0<x<1 (%g", h.Gamma);
  if (h.Lambda <= 0 || h.Lambda > 1) return num("Invalid lambda value, should be in range 0<x<1 (%g", h.Lambda);
  if (h.Epsilon <= 0 || h.Epsilon > 1) return num("Invalid epslion value, should be in range 0<x<1 (%g", h.Epsilon);
  if (h.LogStandardDeviation <= -5 || h.LogStandardDeviation >= 5)
    return num("Invalid log standard deviation value, should be in range -5<x<5 (%g", h.LogStandardDeviation);
  return "";
}

std::string to_json(const Fields& f) {
  std::string o = "{\n";
  bool first = true;
  auto key = [&](const char* k) {
    if (!first) o += ",\n";
    first = false;
    o += std::string("  \"") + k + "\": ";
  };
  auto i = [&](const char* k, int v) { key(k); o += std::to_string(v); };
  auto b = [&](const char* k, int v) { key(k); o += v ? "true" : "false"; };
  auto s = [&](const char* k, const std::string& v) { key(k); o += "\"" + wk::json_escape(v) + "\""; };
  auto f32 = [&](const char* k, float v) { key(k); o += wk::dotnet_float(v, true); };
  i("GameSpeed", f.GameSpeed); b("CollectData", f.CollectData); b("SaveWeights", f.SaveWeights);
  i("Iterations", f.Iterations); i("MaxTimesteps", f.MaxTimesteps); b("RoughFloor", f.RoughFloor);
  s("CriticNeuralNetwork", f.CriticNeuralNetwork); s("ActorNeuralNetwork", f.ActorNeuralNetwork);
  s("CriticWeightFileName", f.CriticWeightFileName); s("ActorWeightFileName", f.ActorWeightFileName);
  s("FilePath", f.FilePath);
  f32("Alpha", f.Alpha); f32("Beta1", f.Beta1); f32("Beta2", f.Beta2); f32("AdamEpsilon", f.AdamEpsilon);
  i("Epochs", f.Epochs); i("BatchSize", f.BatchSize); b("UseGAE", f.UseGAE);
  b("NormalizeAdvantages", f.NormalizeAdvantages);
  f32("Gamma", f.Gamma); f32("Lambda", f.Lambda); f32("Epsilon", f.Epsilon);
  f32("LogStandardDeviation", f.LogStandardDeviation);
  return o + "\n}";
}

bool read_text(const char* path, std::string& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  char buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, k);
  fclose(f);
  return true;
}

}  // namespace

extern "C" {

void wk_host_settings_defaults(wk_host_settings* h) {
  if (!h) return;
  memset(h, 0, sizeof(*h));
  h->CollectData = 1;
  h->SaveWeights = 1;
  copy_str(h->CriticNeuralNetwork, sizeof h->CriticNeuralNetwork, kCriticDefault);
  copy_str(h->ActorNeuralNetwork, sizeof h->ActorNeuralNetwork, kActorDefault);
  copy_str(h->CriticWeightFileName, sizeof h->CriticWeightFileName, "critic");
  copy_str(h->ActorWeightFileName, sizeof h->ActorWeightFileName, "actor");
  copy_str(h->FilePath, sizeof h->FilePath, base_directory());
}

int wk_config_to_json(const wk_config* cfg, const wk_host_settings* host, char* out, size_t cap) {
  wk_config c;
  wk_host_settings h;
  if (cfg) c = *cfg; else wk_config_defaults(&c);
  if (host) h = *host; else wk_host_settings_defaults(&h);
  const Fields f = from(&c, &h);
  for (float v : {f.Alpha, f.Beta1, f.Beta2, f.AdamEpsilon, f.Gamma, f.Lambda, f.Epsilon, f.LogStandardDeviation})
    if (!std::isfinite(v)) {  // JsonSerializer refuses NaN / infinity by default
      wk::set_last_error(".NET number values such as positive and negative infinity cannot be written as valid JSON.");
      return WK_ERR_ARG;
    }
  const std::string j = to_json(f);
  if (!out || cap < j.size() + 1) return -(int)(j.size() + 1);
  memcpy(out, j.c_str(), j.size() + 1);
  return WK_OK;
}

int wk_config_from_json(const char* json, wk_config* cfg, wk_host_settings* host) {
  if (!json || !cfg || !host) { wk::set_last_error("null argument"); return WK_ERR_ARG; }
  wk::JsonValue root;
  std::string why;
  if (!wk::json_parse(json, root, why)) {
    wk::set_last_error("JSON deserializer error. (" + why + ")");
    return WK_ERR_CONFIG;
  }
  Fields f = from(cfg, host);
  if (root.kind == wk::JsonValue::Object) {
    struct Slot { const char* name; int* i; int* b; float* f; std::string* s; bool* isnull; };
    const Slot slots[] = {
        {"GameSpeed", &f.GameSpeed}, {"CollectData", nullptr, &f.CollectData},
        {"SaveWeights", nullptr, &f.SaveWeights}, {"Iterations", &f.Iterations},
        {"MaxTimesteps", &f.MaxTimesteps}, {"RoughFloor", nullptr, &f.RoughFloor},
        {"CriticNeuralNetwork", nullptr, nullptr, nullptr, &f.CriticNeuralNetwork, &f.critic_null},
        {"ActorNeuralNetwork", nullptr, nullptr, nullptr, &f.ActorNeuralNetwork, &f.actor_null},
        {"CriticWeightFileName", nullptr, nullptr, nullptr, &f.CriticWeightFileName, &f.cname_null},
        {"ActorWeightFileName", nullptr, nullptr, nullptr, &f.ActorWeightFileName, &f.aname_null},
        {"FilePath", nullptr, nullptr, nullptr, &f.FilePath, &f.path_null},
        {"Alpha", nullptr, nullptr, &f.Alpha}, {"Beta1", nullptr, nullptr, &f.Beta1},
        {"Beta2", nullptr, nullptr, &f.Beta2}, {"AdamEpsilon", nullptr, nullptr, &f.AdamEpsilon},
        {"Epochs", &f.Epochs}, {"BatchSize", &f.BatchSize}, {"UseGAE", nullptr, &f.UseGAE},
        {"NormalizeAdvantages", nullptr, &f.NormalizeAdvantages},
        {"Gamma", nullptr, nullptr, &f.Gamma}, {"Lambda", nullptr, nullptr, &f.Lambda},
        {"Epsilon", nullptr, nullptr, &f.Epsilon},
        {"LogStandardDeviation", nullptr, nullptr, &f.LogStandardDeviation},
    };
    for (const auto& m : root.members) {
      const wk::JsonValue& v = m.second;
      for (const Slot& sl : slots) {
        if (m.first != sl.name) continue;  // case-sensitive; unknown names are ignored
        bool ok;
        const char* type;
        if (sl.i) { type = "System.Int32"; ok = get_int(v, *sl.i); }
        else if (sl.b) {
          type = "System.Boolean";
          ok = v.kind == wk::JsonValue::Bool;
          if (ok) *sl.b = v.b;
        } else if (sl.f) { type = "System.Single"; ok = get_float(v, *sl.f); }
        else {
          type = "System.String";
          ok = v.kind == wk::JsonValue::String || v.kind == wk::JsonValue::Null;
          if (ok) { *sl.s = v.text; *sl.isnull = v.kind == wk::JsonValue::Null; }
        }
        if (!ok) {
          wk::set_last_error("JSON deserializer error. (The JSON value could not be converted to " +
                             std::string(type) + ". Path: $." + m.first + ")");
          return WK_ERR_CONFIG;
        }
      }
    }
  } else if (root.kind != wk::JsonValue::Null) {
    wk::set_last_error("JSON deserializer error. (The JSON value could not be converted to "
                       "NEA.Walker.PPO.SerializableHyperparameters. Path: $)");
    return WK_ERR_CONFIG;
  }
  if (root.kind == wk::JsonValue::Object) {
    const std::string bad = validate_values(f);
    if (!bad.empty()) {
      wk::set_last_error("Exception occurred while setting the values of the hyperparameters "
                         "during deserialization: (" + bad + ")");
      return WK_ERR_CONFIG;
    }
    cfg->GameSpeed = f.GameSpeed; host->CollectData = f.CollectData; host->SaveWeights = f.SaveWeights;
    cfg->Iterations = f.Iterations; cfg->RoughFloor = f.RoughFloor; cfg->MaxTimesteps = f.MaxTimesteps;
    cfg->Alpha = f.Alpha; cfg->Beta1 = f.Beta1; cfg->Beta2 = f.Beta2; cfg->AdamEpsilon = f.AdamEpsilon;
    cfg->Epochs = f.Epochs; cfg->BatchSize = f.BatchSize <= 0 ? 64 : f.BatchSize;
    cfg->UseGAE = f.UseGAE; cfg->NormalizeAdvantages = f.NormalizeAdvantages;
    cfg->Gamma = f.Gamma; cfg->Lambda = f.Lambda; cfg->Epsilon = f.Epsilon;
    cfg->LogStandardDeviation = f.LogStandardDeviation;
  } else {  // a JSON null document changes nothing; the variables are still validated
    f.critic_null = f.actor_null = f.cname_null = f.aname_null = f.path_null = false;
  }
  // ValidateVariables (Hyperparameters.cs:240-290)
  std::string log;
  int fixes = 0;
  auto report = [&](const std::string& m) { log += (log.empty() ? "" : "\n") + m; fixes++; };
  if (f.path_null || !valid_file_path(f.FilePath.c_str())) {
    report("Invalid file path for the program. (file path is invalid)");
    f.FilePath = base_directory();
    f.path_null = false;
  }
  const bool cname_ok = !f.cname_null && valid_file_name(f.CriticWeightFileName.c_str());
  const bool aname_ok = !f.aname_null && valid_file_name(f.ActorWeightFileName.c_str());
  if (!cname_ok || !aname_ok) {
    std::string ea = aname_ok ? "" : "actor weights file name is invalid";
    std::string ec = cname_ok ? "" : "critic weights file name is invalid";
    if (!aname_ok) f.ActorWeightFileName = "actor";
    if (!cname_ok) f.CriticWeightFileName = "critic";
    report("Invalid file names. (" + ea + (!aname_ok && !cname_ok ? "; " : "") + ec + ")");
  }
  std::string wc, wa;
  const bool c_ok = !f.critic_null && valid_network(f.CriticNeuralNetwork.c_str(), true, wc);
  const bool a_ok = !f.actor_null && valid_network(f.ActorNeuralNetwork.c_str(), false, wa);
  if (f.critic_null) wc = "neural network not valid, check syntax";
  if (f.actor_null) wa = "neural network not valid, check syntax";
  if (!c_ok || !a_ok) {
    if (!a_ok) f.ActorNeuralNetwork = kActorDefault;
    if (!c_ok) f.CriticNeuralNetwork = kCriticDefault;
    report("Invalid neural networks. " + (a_ok ? std::string() : "actor " + wa) +
           (!a_ok && !c_ok ? "; " : "") + (c_ok ? std::string() : "critic " + wc));
  }
  copy_str(host->CriticNeuralNetwork, sizeof host->CriticNeuralNetwork, f.CriticNeuralNetwork);
  copy_str(host->ActorNeuralNetwork, sizeof host->ActorNeuralNetwork, f.ActorNeuralNetwork);
  copy_str(host->CriticWeightFileName, sizeof host->CriticWeightFileName, f.CriticWeightFileName);
  copy_str(host->ActorWeightFileName, sizeof host->ActorWeightFileName, f.ActorWeightFileName);
  copy_str(host->FilePath, sizeof host->FilePath, f.FilePath);
  cfg->CriticNeuralNetwork = host->CriticNeuralNetwork;
  cfg->ActorNeuralNetwork = host->ActorNeuralNetwork;
  wk::set_last_error(log);
  return fixes;
}

int wk_config_save_json(const char* path, const wk_config* cfg, const wk_host_settings* host) {
  if (!path) { wk::set_last_error("null path"); return WK_ERR_ARG; }
  const int need = -wk_config_to_json(cfg, host, nullptr, 0);
  if (need <= 0) return need == 0 ? WK_ERR_ARG : -need;
  std::string buf((size_t)need, '\0');
  const int r = wk_config_to_json(cfg, host, &buf[0], buf.size());
  if (r != WK_OK) return r;
  FILE* f = fopen(path, "wb");
  if (!f) { wk::set_last_error(std::string("cannot write '") + path + "'"); return WK_ERR_ARG; }
  const size_t n = strlen(buf.c_str());
  const bool ok = fwrite(buf.data(), 1, n, f) == n;
  if (fclose(f) != 0 || !ok) { wk::set_last_error(std::string("cannot write '") + path + "'"); return WK_ERR_ARG; }
  return WK_OK;
}

int wk_config_load_json(const char* path, wk_config* cfg, wk_host_settings* host) {
  std::string text;
  if (!path || !read_text(path, text)) {
    wk::set_last_error(std::string("cannot read '") + (path ? path : "(null)") + "'");
    return WK_ERR_ARG;
  }
  if (text.find('\0') != std::string::npos) {
    wk::set_last_error("JSON deserializer error. (NUL byte in the document)");
    return WK_ERR_CONFIG;
  }
  return wk_config_from_json(text.c_str(), cfg, host);
}

}  // extern "C"
