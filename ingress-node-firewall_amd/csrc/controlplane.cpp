// controlplane.cpp — byte encoders of the table map contract, restating the
// Go helpers the reference's loader writes the map with:
//   BuildEBPFKey           pkg/ebpf/ingress_node_firewall_loader.go:530-547
//   makeIngressFwRulesMap  pkg/ebpf/ingress_node_firewall_loader.go:429-515
//   IsRange/GetPort/GetRange  pkg/utils/utils.go:13-60
// CIDR parsing follows Go 1.18+ net.ParseCIDR (netip.ParseAddr for the
// address, decimal mask 0..BitLen, no zones).
#include <errno.h>
#include <string.h>

#include <string>

#include "infw_internal.h"

namespace {

bool parse_v4(const char *s, size_t n, uint8_t out[4]) {
    // netip.parseIPv4: exactly 4 decimal fields, each <= 255, no leading zeros
    int field = 0;
    size_t i = 0;
    while (field < 4) {
        if (i >= n || s[i] < '0' || s[i] > '9') return false;
        size_t st = i;
        uint32_t v = 0;
        while (i < n && s[i] >= '0' && s[i] <= '9') {
            v = v * 10 + (uint32_t)(s[i] - '0');
            if (v > 255) return false;
            i++;
        }
        if (i - st > 1 && s[st] == '0') return false;
        out[field++] = (uint8_t)v;
        if (field < 4) {
            if (i >= n || s[i] != '.') return false;
            i++;
        }
    }
    return i == n;
}

int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

bool parse_v6(const char *s, size_t n, uint8_t out[16]) {
    // netip.parseIPv6: groups of 1-4 hex digits, one "::" ellipsis, optional
    // trailing dotted IPv4, no zone.
    uint8_t ip[16] = {0};
    int ellipsis = -1, k = 0;
    size_t i = 0;
    if (n >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0;
        i = 2;
        if (i == n) {
            memset(out, 0, 16);
            return true;
        }
    }
    while (k < 16) {
        size_t st = i;
        uint32_t acc = 0;
        int nd = 0;
        while (i < n && hexval(s[i]) >= 0) {
            acc = acc * 16 + (uint32_t)hexval(s[i]);
            i++;
            nd++;
            if (nd > 4) return false;
        }
        if (nd == 0) return false;
        if (i < n && s[i] == '.') {  // embedded IPv4 in the last 32 bits
            if (ellipsis < 0 && k != 12) return false;
            if (k + 4 > 16) return false;
            uint8_t v4[4];
            if (!parse_v4(s + st, n - st, v4)) return false;
            memcpy(ip + k, v4, 4);
            k += 4;
            i = n;
            break;
        }
        ip[k] = (uint8_t)(acc >> 8);
        ip[k + 1] = (uint8_t)acc;
        k += 2;
        if (i == n) break;
        if (s[i] != ':' || i + 1 == n) return false;
        i++;
        if (s[i] == ':') {
            if (ellipsis >= 0) return false;
            ellipsis = k;
            i++;
            if (i == n) break;
        }
    }
    if (i != n) return false;
    if (k < 16) {
        if (ellipsis < 0) return false;
        int nmove = k - ellipsis;
        for (int j = nmove - 1; j >= 0; j--) ip[16 - nmove + j] = ip[ellipsis + j];
        for (int j = ellipsis; j < 16 - nmove; j++) ip[j] = 0;
    } else if (ellipsis >= 0) {
        return false;  // "::" must stand for at least one group
    }
    memcpy(out, ip, 16);
    return true;
}

// strconv.ParseUint(s, 10, 16): decimal digits only, value <= 65535
bool parse_u16(const std::string &s, uint32_t *v) {
    if (s.empty()) return false;
    uint64_t acc = 0;
    for (char c : s) {
        if (c < '0' || c > '9') return false;
        acc = acc * 10 + (uint64_t)(c - '0');
        if (acc > 0xFFFF) return false;
    }
    *v = (uint32_t)acc;
    return true;
}

}  // namespace

extern "C" {

int infw_build_ebpf_key(uint32_t if_id, const char *cidr, lpm_ip_key_st *key) {
    if (!cidr || !key) return -EINVAL;
    memset(key, 0, sizeof(*key));
    const char *slash = strchr(cidr, '/');
    if (!slash) {
        infw::set_error("Failed to parse SourceCIDRs: missing '/'");
        return -EINVAL;
    }
    size_t alen = (size_t)(slash - cidr);
    uint8_t ip16[16];
    int bitlen;
    uint8_t v4[4];
    if (parse_v4(cidr, alen, v4)) {
        memset(ip16, 0, 10);
        ip16[10] = ip16[11] = 0xFF;
        memcpy(ip16 + 12, v4, 4);
        bitlen = 32;
    } else if (parse_v6(cidr, alen, ip16)) {
        bitlen = 128;
    } else {
        infw::set_error(std::string("Failed to parse SourceCIDRs: bad address in ") + cidr);
        return -EINVAL;
    }
    // dtoi: decimal, leading zeros allowed, must consume the rest
    const char *m = slash + 1;
    if (!*m) {
        infw::set_error("Failed to parse SourceCIDRs: empty mask");
        return -EINVAL;
    }
    uint32_t mask = 0;
    for (const char *p = m; *p; p++) {
        if (*p < '0' || *p > '9') {
            infw::set_error("Failed to parse SourceCIDRs: bad mask");
            return -EINVAL;
        }
        mask = mask * 10 + (uint32_t)(*p - '0');
        if (mask > 0xFFFFFF) {
            infw::set_error("Failed to parse SourceCIDRs: mask too large");
            return -EINVAL;
        }
    }
    if ((int)mask > bitlen) {
        infw::set_error("Failed to parse SourceCIDRs: mask exceeds address length");
        return -EINVAL;
    }
    // loader.go:537-541: ip.To4() != nil (an IPv4 or IPv4-mapped address) copies 4 bytes
    static const uint8_t v4mapped[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xFF, 0xFF};
    if (memcmp(ip16, v4mapped, 12) == 0) memcpy(key->ip_data, ip16 + 12, 4);
    else memcpy(key->ip_data, ip16, 16);
    key->prefixLen = mask + 32;  // pfLen + ifIndexKeyLength (loader.go:542-543)
    key->ingress_ifindex = if_id;
    return 0;
}

int infw_make_rule(rulesVal_st *val, uint32_t order, const char *protocol, const char *ports,
                   uint8_t icmp_type, uint8_t icmp_code, const char *action) {
    if (!val) return -EINVAL;
    if (order >= INFW_MAX_RULES_PER_TARGET) {
        infw::set_error("order out of range of rulesVal_st.rules (loader.go:437 would panic)");
        return -E2BIG;
    }
    ruleType_st &r = val->rules[order];
    r.ruleId = order;  // loader.go:438
    std::string proto = protocol ? protocol : "";
    if (proto == "TCP" || proto == "UDP" || proto == "SCTP") {
        if (!ports) {
            infw::set_error("transport rule without ports (nil ProtocolConfig pointer in Go)");
            return -EINVAL;
        }
        std::string p = ports;
        if (p.find('-') != std::string::npos) {  // IsRange, utils.go:13-18
            size_t dash = p.find('-');
            uint32_t start, end;
            if (!parse_u16(p.substr(0, dash), &start) || !parse_u16(p.substr(dash + 1), &end)) {
                infw::set_error("invalid Port range " + p);
                return -EINVAL;
            }
            if (start > end || start == end || start == 0) {  // utils.go:50-58
                infw::set_error("invalid Port range " + p);
                return -EINVAL;
            }
            r.dstPortStart = (uint16_t)start;
            r.dstPortEnd = (uint16_t)end;  // stored as typed; the data path treats it as exclusive
        } else {
            uint32_t port;
            if (!parse_u16(p, &port) || port == 0) {  // utils.go:24-30
                infw::set_error("invalid Port " + p);
                return -EINVAL;
            }
            r.dstPortStart = (uint16_t)port;
            r.dstPortEnd = 0;
        }
        r.protocol = proto == "TCP" ? 6 : proto == "UDP" ? 17 : 132;
    } else if (proto == "ICMP") {
        r.icmpType = icmp_type;
        r.icmpCode = icmp_code;
        r.protocol = 1;
    } else if (proto == "ICMPv6") {
        r.icmpType = icmp_type;
        r.icmpCode = icmp_code;
        r.protocol = 58;
    }
    // any other protocol string: no case in the Go switch, fields untouched (protocol 0)
    std::string act = action ? action : "";
    if (act == "Allow") r.action = INFW_XDP_PASS;       // xdpAllow = 2 (loader.go:31)
    else if (act == "Deny") r.action = INFW_XDP_DROP;   // xdpDeny = 1 (loader.go:30)
    else {
        infw::set_error("Failed invalid action " + act);
        return -EINVAL;
    }
    return 0;
}

}  // extern "C"
