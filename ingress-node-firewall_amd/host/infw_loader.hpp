// infw_loader.hpp — host side above the C ABI, in C++: the reference's map-population API (pkg/ebpf
// IngNodeFwController) and statistics reader (pkg/metrics), driving libinfw instead of an *ebpf.Map.
//
// The reference's host side is Go (compiled); Go is not in this image, so this is the C++ form a daemon links
// (INTEGRATION.md shows the cgo binding that would replace it when Go is present).  Same names, argument meaning
// and error behaviour as the Go code:
//   IngNodeFwController::IngressNodeFwRulesLoader   loader.go:130-194
//   IngNodeFwController::MakeIngressFwRulesMap      loader.go:429-527 (BuildEBPFKey :530-547 via the C ABI)
//   IngNodeFwController::GetStaleKeys / PurgeKeys / AddOrUpdateRules
//                                                   loader.go:551-581, 633-649, 200-208
//   IngNodeFwController::GetBPFMapContentForTest    loader.go:286-303
//   IngNodeFwController::ResetAll                   ebpfsyncer.go:160-178 (the table map dropped with the objects)
//   UpdateMetrics / AddUInt64                       statistics.go:112-180
// Errors are negative errnos (bpf(2) style, what the Go code wraps); the message of the last failing C ABI call is
// in infw_last_error().  Interface names are resolved by caller-supplied functions (the reference uses netlink,
// pkg/interfaces/interfaces.go:85-116 — out of scope).
#pragma once
#include <stdint.h>

#include <array>
#include <functional>
#include <map>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "../../include/infw.h"

namespace infw {
namespace loader {

// IngressNodeFirewallProtocolRule (api/v1alpha1/ingressnodefirewall_types.go:91-107).
struct ProtocolRule {
    uint32_t order = 0;
    std::string protocol;              // "TCP" | "UDP" | "SCTP" | "ICMP" | "ICMPv6" | "" (no protocolConfig)
    std::optional<std::string> ports;  // intstr: "80" or "100-200"
    uint8_t icmp_type = 0, icmp_code = 0;
    std::string action = "Allow";
};

// IngressNodeFirewallRules (ingressnodefirewall_types.go:139-147).
struct IngressNodeFirewallRules {
    std::vector<std::string> source_cidrs;
    std::vector<ProtocolRule> rules;
};

// map[string][]IngressNodeFirewallRules, in the caller's order (a Go map range has none).
using InterfaceRules = std::vector<std::pair<std::string, std::vector<IngressNodeFirewallRules>>>;

using KeyBytes = std::array<uint8_t, sizeof(lpm_ip_key_st)>;
KeyBytes key_bytes(const lpm_ip_key_st &k);

// strconv.Atoi: optional sign, decimal digits only, int64 range; false where Go returns an error.
bool go_atoi(const std::string &s, int64_t *out);

class IngNodeFwController {
  public:
    using IfIndices = std::function<int(const std::string &, std::vector<uint32_t> *)>;  // GetInterfaceIndices
    using IsValid = std::function<bool(const std::string &)>;                           // IsValidInterfaceNameAndState

    // ENABLE_EBPF_LPM_LOOKUP_DBG sets the debug_lookup constant (loader.go:72-83); `env_debug_lookup` is its
    // value (nullptr: unset).  *rc < 0 when it is not an integer (the Go code fails the load there).
    IngNodeFwController(infw_ctx *ctx, IfIndices if_indices, IsValid is_valid, const char *env_debug_lookup,
                        int *rc);

    // loader.go:130-194: build the desired key -> value map (last writer wins), purge the stale keys (errors are
    // collected in *purge_errors, not fatal), add or update every desired key, publish the epoch.  An update error
    // ends the load like the Go code's, and the updates made before it are published (the reference's per-key map
    // writes are live at once).
    int IngressNodeFwRulesLoader(const InterfaceRules &iface_rules, std::vector<int> *purge_errors = nullptr);

    // loader.go:429-527: one value for the rule set, one key per source CIDR.
    int MakeIngressFwRulesMap(const IngressNodeFirewallRules &cfg, uint32_t if_id, std::vector<lpm_ip_key_st> *keys,
                              rulesVal_st *val) const;
    // loader.go:551-581, in O(N) (the reference compares every map key with every desired key).
    int GetStaleKeys(const std::vector<lpm_ip_key_st> &desired, std::vector<lpm_ip_key_st> *stale) const;
    // loader.go:633-649: every key is tried; the failures are returned.
    std::vector<int> PurgeKeys(const std::vector<lpm_ip_key_st> &keys);
    // loader.go:200-208: stops at the first failing update.
    int AddOrUpdateRules(const std::vector<std::pair<lpm_ip_key_st, const rulesVal_st *>> &key_to_rules);
    // loader.go:286-303: the committed map, key -> value.
    int GetBPFMapContentForTest(std::map<KeyBytes, rulesVal_st> *out) const;
    int ResetAll();

  private:
    infw_ctx *ctx_;
    IfIndices if_indices_;
    IsValid is_valid_;
};

// statistics.go:170-180: wrap-around sum and whether it is kept.
std::pair<uint64_t, bool> AddUInt64(uint64_t a, uint64_t b);

struct Metrics {
    uint64_t allow_total = 0, allow_bytes = 0, deny_total = 0, deny_bytes = 0;
    uint32_t failed_lookups = 0;  // rules whose statistics read failed (skipped, as statistics.go:127-130 does)
    int last_error = 0;           // the last such read's errno (negative)
};
// statistics.go:112-167: rules 1..MAX_INGRESS_RULES-1, every slot (one per device, like one per CPU).  A failed read
// of one rule is counted in failed_lookups and skipped; -EINVAL only for a null context or output.
int UpdateMetrics(infw_ctx *ctx, Metrics *out);

}  // namespace loader
}  // namespace infw
