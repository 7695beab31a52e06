// YAML (the subset master configs use) -> Json, and the master-config layering the reference does
// with viper (master/cmd/determined-master/root.go:20, master/internal/config.go:24-86):
//   defaults < config file (YAML or JSON; /etc/determined/master.yaml when present) < DET_* env < flags.
//
// Supported YAML: block mappings and sequences (incl. "- key: v" items with continuation keys),
// flow collections ([a, b], {k: v}) nested, plain / 'single' / "double" (escapes) scalars, literal
// (|) and folded (>) block scalars, comments, a leading "---".  Plain scalars resolve like yaml.v2
// (YAML 1.1 core): true/false/yes/no/on/off, null/~, ints (dec, 0x, 0o), floats.  No anchors,
// aliases, tags or multi-document streams.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "detcore/json.h"

namespace detcore {

class YamlError : public std::runtime_error {
 public:
  explicit YamlError(const std::string& m) : std::runtime_error(m) {}
};

Json ParseYaml(const std::string& text);
// One scalar with YAML resolution rules (env values, flag values).
Json YamlScalar(const std::string& text);

// viper-style environment overlay: for every leaf path a.b.c of `schema` (and every extra path in
// `extra_paths`), DET_A_B_C (upper-cased, '-' and '.' -> '_') overrides it when set in `env`.
Json EnvOverlay(const Json& schema, const std::vector<std::string>& extra_paths,
                const std::map<std::string, std::string>& env);

}  // namespace detcore
