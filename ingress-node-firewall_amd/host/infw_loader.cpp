// infw_loader.cpp — see infw_loader.hpp (pkg/ebpf IngNodeFwController and pkg/metrics over libinfw's C ABI).
#include "infw_loader.hpp"

#include <errno.h>
#include <string.h>

#include <unordered_map>
#include <unordered_set>

namespace infw {
namespace loader {

namespace {

struct KeyHash {
    size_t operator()(const KeyBytes &k) const {
        uint64_t h = 0xcbf29ce484222325ull;
        for (uint8_t b : k) h = (h ^ b) * 0x100000001b3ull;
        return (size_t)h;
    }
};

lpm_ip_key_st key_of(const KeyBytes &b) {
    lpm_ip_key_st k;
    memcpy(&k, b.data(), sizeof k);
    return k;
}

constexpr uint32_t kMaxIngressRules = 100;  // pkg/failsaferules MAX_INGRESS_RULES

}  // namespace

KeyBytes key_bytes(const lpm_ip_key_st &k) {
    KeyBytes b;
    memcpy(b.data(), &k, sizeof k);
    return b;
}

bool go_atoi(const std::string &s, int64_t *out) {
    size_t i = (!s.empty() && (s[0] == '+' || s[0] == '-')) ? 1 : 0;
    if (i == s.size()) return false;
    const bool neg = s[0] == '-';
    uint64_t v = 0;
    for (; i < s.size(); i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        const uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (UINT64_MAX - d) / 10) return false;
        v = v * 10 + d;
        if (v > (neg ? (uint64_t)INT64_MAX + 1 : (uint64_t)INT64_MAX)) return false;  // value out of range
    }
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return true;
}

IngNodeFwController::IngNodeFwController(infw_ctx *ctx, IfIndices if_indices, IsValid is_valid,
                                         const char *env_debug_lookup, int *rc)
    : ctx_(ctx), if_indices_(std::move(if_indices)), is_valid_(std::move(is_valid)) {
    int r = 0;
    if (env_debug_lookup) {  // loader.go:72-83: strconv.Atoi, then uint32(...) into the program's constant
        int64_t v = 0;
        r = go_atoi(env_debug_lookup, &v) ? infw_debug_lookup_set(ctx_, (uint32_t)v) : -EINVAL;
    }
    if (rc) *rc = r;
}

int IngNodeFwController::MakeIngressFwRulesMap(const IngressNodeFirewallRules &cfg, uint32_t if_id,
                                               std::vector<lpm_ip_key_st> *keys, rulesVal_st *val) const {
    memset(val, 0, sizeof *val);
    for (const ProtocolRule &r : cfg.rules) {
        const int rc = infw_make_rule(val, r.order, r.protocol.c_str(), r.ports ? r.ports->c_str() : nullptr,
                                      r.icmp_type, r.icmp_code, r.action.c_str());
        if (rc) return rc;
    }
    keys->clear();
    for (const std::string &cidr : cfg.source_cidrs) {
        lpm_ip_key_st k;
        const int rc = infw_build_ebpf_key(if_id, cidr.c_str(), &k);
        if (rc) return rc;
        keys->push_back(k);
    }
    return 0;
}

int IngNodeFwController::IngressNodeFwRulesLoader(const InterfaceRules &iface_rules, std::vector<int> *purge_errors) {
    // the desired key -> value map, in first-insertion order with the last writer's value (loader.go:141-164)
    std::vector<std::pair<KeyBytes, rulesVal_st>> desired;
    std::unordered_map<KeyBytes, size_t, KeyHash> at;
    std::vector<lpm_ip_key_st> keys;
    rulesVal_st val;
    for (const auto &iface : iface_rules) {
        if (is_valid_ && !is_valid_(iface.first)) continue;  // loader.go:143-146
        std::vector<uint32_t> if_ids;                        // bond -> its slaves' indices (loader.go:149)
        int rc = if_indices_(iface.first, &if_ids);
        if (rc) return rc;
        for (const IngressNodeFirewallRules &rule : iface.second)
            for (uint32_t if_id : if_ids) {
                rc = MakeIngressFwRulesMap(rule, if_id, &keys, &val);
                if (rc) return rc;  // "failed to create map firewall rules" (loader.go:160-162)
                for (const lpm_ip_key_st &k : keys) {
                    const KeyBytes kb = key_bytes(k);
                    auto it = at.find(kb);
                    if (it == at.end()) {
                        at.emplace(kb, desired.size());
                        desired.emplace_back(kb, val);
                    } else {
                        desired[it->second].second = val;
                    }
                }
            }
    }
    std::vector<lpm_ip_key_st> want, stale;
    want.reserve(desired.size());
    for (const auto &d : desired) want.push_back(key_of(d.first));
    int rc = GetStaleKeys(want, &stale);
    if (rc) return rc;
    std::vector<int> errs = PurgeKeys(stale);  // logged, not fatal (loader.go:183-186)
    if (purge_errors) *purge_errors = std::move(errs);
    std::vector<std::pair<lpm_ip_key_st, const rulesVal_st *>> updates;
    updates.reserve(desired.size());
    for (size_t i = 0; i < desired.size(); i++) updates.emplace_back(want[i], &desired[i].second);
    rc = AddOrUpdateRules(updates);
    const int crc = infw_table_commit(ctx_);  // publish as one epoch (also what an update error leaves applied)
    return rc ? rc : crc;
}

int IngNodeFwController::GetStaleKeys(const std::vector<lpm_ip_key_st> &desired,
                                      std::vector<lpm_ip_key_st> *stale) const {
    std::unordered_set<KeyBytes, KeyHash> want;
    want.reserve(desired.size() * 2);
    for (const lpm_ip_key_st &k : desired) want.insert(key_bytes(k));
    stale->clear();
    lpm_ip_key_st cur, next;
    const lpm_ip_key_st *prev = nullptr;
    for (;;) {
        const int rc = infw_table_get_next_key(ctx_, prev, &next);
        if (rc == -ENOENT) break;
        if (rc) return rc;
        if (!want.count(key_bytes(next))) stale->push_back(next);
        cur = next;
        prev = &cur;
    }
    return 0;
}

std::vector<int> IngNodeFwController::PurgeKeys(const std::vector<lpm_ip_key_st> &keys) {
    std::vector<int> errs;
    for (const lpm_ip_key_st &k : keys) {
        const int rc = infw_table_delete(ctx_, &k);
        if (rc < 0) errs.push_back(rc);
    }
    return errs;
}

int IngNodeFwController::AddOrUpdateRules(const std::vector<std::pair<lpm_ip_key_st, const rulesVal_st *>> &key_to_rules) {
    for (const auto &kv : key_to_rules) {
        const int rc = infw_table_update(ctx_, &kv.first, kv.second, INFW_BPF_ANY);
        if (rc) return rc;  // "Failed Adding/Updating ingress firewall rules" (loader.go:203-205)
    }
    return 0;
}

int IngNodeFwController::GetBPFMapContentForTest(std::map<KeyBytes, rulesVal_st> *out) const {
    out->clear();
    lpm_ip_key_st cur, next;
    const lpm_ip_key_st *prev = nullptr;
    for (;;) {
        int rc = infw_table_get_next_key(ctx_, prev, &next);
        if (rc == -ENOENT) return 0;
        if (rc) return rc;
        rulesVal_st v;
        rc = infw_table_lookup(ctx_, &next, &v);
        if (rc == 0) (*out)[key_bytes(next)] = v;
        else if (rc != -ENOENT) return rc;
        cur = next;
        prev = &cur;
    }
}

int IngNodeFwController::ResetAll() {
    std::vector<lpm_ip_key_st> all;
    int rc = GetStaleKeys({}, &all);  // every key is stale against an empty desired set
    if (rc) return rc;
    for (const lpm_ip_key_st &k : all) {
        rc = infw_table_delete(ctx_, &k);
        if (rc) return rc;
    }
    rc = infw_table_commit(ctx_);
    if (rc) return rc;
    // resetAll closes the objects (ebpfsyncer.go:170), the statistics map with them: the next load counts from zero
    return infw_stats_reset(ctx_);
}

std::pair<uint64_t, bool> AddUInt64(uint64_t a, uint64_t b) {
    const uint64_t c = a + b;
    if (a == 0 || b == 0) return {c, true};
    if (c > a && c > b) return {c, true};
    return {c, false};
}

int UpdateMetrics(infw_ctx *ctx, Metrics *out) {
    if (!ctx || !out) return -EINVAL;
    *out = Metrics{};
    const int nd = infw_num_devices(ctx);
    std::vector<ruleStatistics_st> slots((size_t)(nd > 0 ? nd : 1));
    for (uint32_t rule = 1; rule < kMaxIngressRules; rule++) {  // statistics.go:126
        int n = 0;
        const int rc = infw_stats_read(ctx, rule, slots.data(), &n);
        if (rc) {  // statistics.go:127-130 logs the failed lookup and goes on with the next rule
            out->failed_lookups++;
            out->last_error = rc;
            continue;
        }
        for (int s = 0; s < n; s++) {  // a sum that wraps is dropped, as addUInt64's callers do (:135-156)
            auto add = [](uint64_t &acc, uint64_t v) {
                const auto r = AddUInt64(v, acc);
                if (r.second) acc = r.first;
            };
            add(out->allow_total, slots[s].allow_stats.packets);
            add(out->allow_bytes, slots[s].allow_stats.bytes);
            add(out->deny_total, slots[s].deny_stats.packets);
            add(out->deny_bytes, slots[s].deny_stats.bytes);
        }
    }
    return 0;
}

}  // namespace loader
}  // namespace infw
