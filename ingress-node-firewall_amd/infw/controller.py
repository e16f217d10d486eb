"""Host-side mirror of the reference's map-population API (pkg/ebpf) and stats
reader (pkg/metrics), driving the GPU backend through libinfw's C ABI.

  IngNodeFwController.ingress_node_fw_rules_loader  loader.go:130-194
  IngNodeFwController.make_ingress_fw_rules_map     loader.go:429-527
  IngNodeFwController.get_stale_keys / purge_keys / add_or_update_rules
                                                     loader.go:551-581, 633-649, 200-208
  IngNodeFwController.get_bpf_map_content_for_test  loader.go:286-303
  Statistics.update_metrics                          statistics.go:112-167

Interface names are resolved by a caller-supplied function (the reference uses
netlink, pkg/interfaces/interfaces.go:85-116 — out of scope here).
"""
from __future__ import annotations

import os

import ctypes as C
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Union

from . import _native as N
from .core import Classifier, build_ebpf_key
from ._native import InfwError, LpmIpKeySt, RulesValSt


@dataclass
class ProtocolRule:
    """IngressNodeFirewallProtocolRule (api/v1alpha1/ingressnodefirewall_types.go:91-107)."""
    order: int
    protocol: str = ""            # "TCP" | "UDP" | "SCTP" | "ICMP" | "ICMPv6" | "" (no protocolConfig)
    ports: Optional[Union[str, int]] = None  # intstr: "80", 80 or "100-200"
    icmp_type: int = 0
    icmp_code: int = 0
    action: str = "Allow"


@dataclass
class IngressNodeFirewallRules:
    """IngressNodeFirewallRules (ingressnodefirewall_types.go:139-147)."""
    source_cidrs: List[str]
    rules: List[ProtocolRule] = field(default_factory=list)


def make_rules_val(rules: Sequence[ProtocolRule]) -> RulesValSt:
    """The rulesVal_st part of makeIngressFwRulesMap (loader.go:435-515)."""
    val = RulesValSt()
    for r in rules:
        ports = None if r.ports is None else str(r.ports).encode()
        rc = N.lib.infw_make_rule(C.byref(val), r.order, r.protocol.encode(), ports, r.icmp_type & 0xFF,
                                  r.icmp_code & 0xFF, r.action.encode())
        N.check(rc, f"makeIngressFwRulesMap(order={r.order})")
    return val


DEBUG_LOOKUP_ENV = "ENABLE_EBPF_LPM_LOOKUP_DBG"


def go_atoi(s: str) -> int:
    """strconv.Atoi: optional sign, decimal digits only, int64 range; ValueError like the Go error."""
    t = s[1:] if s[:1] in "+-" else s
    if not t or not t.isascii() or not t.isdigit():
        raise ValueError(f'failed to convert "{s}" to integer: strconv.Atoi: parsing "{s}": invalid syntax')
    v = int(s)
    if not -(1 << 63) <= v < (1 << 63):
        raise ValueError(f'failed to convert "{s}" to integer: strconv.Atoi: parsing "{s}": value out of range')
    return v


class IngNodeFwController:
    """IngNodeFwController (loader.go:43-50) with the table map on the GPU."""

    def __init__(self, classifier: Classifier, if_indices: Callable[[str], List[int]],
                 is_valid_interface: Callable[[str], bool] = lambda name: True, environ=None):
        self.c = classifier
        self.if_indices = if_indices
        self.is_valid_interface = is_valid_interface
        # debug_lookup constant from ENABLE_EBPF_LPM_LOOKUP_DBG (loader.go:37-38, :72-83)
        env = os.environ if environ is None else environ
        if DEBUG_LOOKUP_ENV in env:
            self.c.debug_lookup(go_atoi(env[DEBUG_LOOKUP_ENV]) & 0xFFFFFFFF)

    def make_ingress_fw_rules_map(self, cfg: IngressNodeFirewallRules, if_id: int):
        val = make_rules_val(cfg.rules)
        keys = [build_ebpf_key(if_id, cidr) for cidr in cfg.source_cidrs]
        return keys, val

    def ingress_node_fw_rules_loader(self, iface_rules: Dict[str, List[IngressNodeFirewallRules]]) -> None:
        key_to_rules: Dict[bytes, RulesValSt] = {}
        for name, ingress_rules in iface_rules.items():
            if not self.is_valid_interface(name):          # loader.go:143-146
                continue
            if_ids = self.if_indices(name)                   # bond -> slaves, loader.go:149
            for rule in ingress_rules:
                for if_id in if_ids:
                    keys, val = self.make_ingress_fw_rules_map(rule, if_id)
                    for k in keys:
                        key_to_rules[bytes(k)] = val         # identical keys: last writer wins
        desired = [LpmIpKeySt.from_buffer_copy(k) for k in key_to_rules]
        stale = self.get_stale_keys(desired)
        errs = self.purge_keys(stale)                        # errors logged, not fatal (loader.go:183-186)
        # an update error (e.g. ENOSPC) ends the load (loader.go:187-188), but the reference's per-key map
        # updates made before it are live: publish them rather than leave them pending for a later commit.
        # The caller sees the update's own error; a commit failure after it is chained as its cause.
        try:
            self.add_or_update_rules(key_to_rules)
        except Exception as update_err:
            try:
                self.c.commit()
            except Exception as commit_err:
                raise update_err from commit_err
            raise
        self.c.commit()                                      # publish as one epoch
        return errs

    def get_stale_keys(self, desired: List[LpmIpKeySt]) -> List[LpmIpKeySt]:
        want = {bytes(k) for k in desired}                   # O(N) instead of O(N*M) DeepEqual
        return [LpmIpKeySt.from_buffer_copy(bytes(k)) for k, _ in self.c.iterate() if bytes(k) not in want]

    def purge_keys(self, keys: List[LpmIpKeySt]) -> List[int]:
        return [rc for rc in (self.c.delete_rc(k) for k in keys) if rc < 0]

    def add_or_update_rules(self, key_to_rules: Dict[bytes, RulesValSt]) -> None:
        for kb, val in key_to_rules.items():
            self.c.update(LpmIpKeySt.from_buffer_copy(kb), val, N.BPF_ANY)

    def get_bpf_map_content_for_test(self) -> Dict[bytes, RulesValSt]:
        return {bytes(k): v for k, v in self.c.iterate()}

    def reset_all(self) -> None:
        """ebpfsyncer resetAll (ebpfsyncer.go:160-178): the table map is dropped with the objects."""
        for k, _ in list(self.c.iterate()):
            self.c.delete(k)
        self.c.commit()
        self.c.stats_reset()  # the statistics map goes with the closed objects (ebpfsyncer.go:170)


def add_uint64(a: int, b: int):
    """addUInt64 (statistics.go:170-180): wrap-around sum and an overflow flag."""
    c = (a + b) & 0xFFFFFFFFFFFFFFFF
    if a == 0 or b == 0:
        return c, True
    if c > a and c > b:
        return c, True
    return c, False


class Statistics:
    """pkg/metrics Statistics: per-rule slots summed for rules 1..MAX_INGRESS_RULES-1."""

    MAX_INGRESS_RULES = 100  # pkg/failsaferules MAX_INGRESS_RULES

    def __init__(self, classifier: Classifier):
        self.c = classifier

    def update_metrics(self) -> Dict[str, int]:
        allow = allow_b = deny = deny_b = 0
        self.failed_lookups = 0
        for rule in range(1, self.MAX_INGRESS_RULES):        # statistics.go:126
            try:
                slots = self.c.stats_read(rule, wait=False)  # a snapshot beside running batches, as XDP runs on
            except InfwError:                                # statistics.go:127-130: logged, next rule
                self.failed_lookups += 1
                continue
            for s in slots:
                v, ok = add_uint64(s.allow_packets, allow)
                allow = v if ok else allow
                v, ok = add_uint64(s.allow_bytes, allow_b)
                allow_b = v if ok else allow_b
                v, ok = add_uint64(s.deny_packets, deny)
                deny = v if ok else deny
                v, ok = add_uint64(s.deny_bytes, deny_b)
                deny_b = v if ok else deny_b
        return {"ingressnodefirewall_node_packet_allow_total": allow,
                "ingressnodefirewall_node_packet_allow_bytes": allow_b,
                "ingressnodefirewall_node_packet_deny_total": deny,
                "ingressnodefirewall_node_packet_deny_bytes": deny_b}
