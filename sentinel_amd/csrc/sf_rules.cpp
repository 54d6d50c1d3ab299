// sf_rules.cpp — the order in which the reference's rule managers iterate a
// resource's rules (product code, host only; the C-ABI helpers
// sf_flow_rule_order / sf_param_rule_order of include/sentinel_flow.h).
//
// FlowRuleUtil.buildFlowRuleMap (FlowRuleUtil.java:83-130): the valid rules
// of a resource go through a java.util.HashSet (an equal rule is dropped),
// the set is copied into a list in HashMap iteration order and sorted stably
// with FlowRuleComparator (FlowRuleComparator.java:27-57).  The ParamFlow
// manager does the same without the sort (ParamFlowRuleUtil.java:138-186).
// A rule that fails first is the one that blocks, and an earlier passing
// ParamFlow rule has already consumed tokens, so this order is part of the
// decisions (SURVEY.md §7 hard part 5).
#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "sf_decide.h"

namespace {

using namespace sf;

int32_t mix(int32_t h, int32_t v) { return (int32_t)((uint32_t)h * 31u + (uint32_t)v); }
int32_t mix_double(int32_t h, double x) {                      // Double.doubleToLongBits
    uint64_t t;
    if (x != x) t = 0x7ff8000000000000ULL;
    else std::memcpy(&t, &x, 8);
    return mix(h, (int32_t)(uint32_t)(t ^ (t >> 32)));
}
bool same_double(double a, double b) {                          // Double.compare == 0
    if (a != a && b != b) return true;
    uint64_t x, y;
    std::memcpy(&x, &a, 8); std::memcpy(&y, &b, 8);
    return x == y;
}

// AbstractRule.hashCode (AbstractRule.java:111-118): limitApp only when not "default"
int32_t abstract_hash(const sf_rule_key& k) {
    int32_t h = k.resource_hash;
    if (k.limit_app_id != 0) h = mix(h, k.limit_app_hash);
    return h;
}
// FlowRule.hashCode (FlowRule.java:207-222); clusterConfig: null
int32_t flow_hash(const sf_flow_rule& r, const sf_rule_key& k) {
    int32_t h = mix(abstract_hash(k), r.grade);
    h = mix_double(h, r.count);
    h = mix(h, r.strategy);
    h = mix(h, k.extra_hash);
    h = mix(h, r.control_behavior);
    h = mix(h, r.warm_up_period_sec);
    h = mix(h, r.max_queueing_time_ms);
    h = mix(h, r.cluster_mode ? 1 : 0);
    return mix(h, k.cluster_hash);
}
// ParamFlowRule.hashCode (ParamFlowRule.java:211-227); clusterMode false, clusterConfig null
int32_t param_hash(const sf_param_rule& r, const sf_rule_key& k) {
    int32_t h = mix(abstract_hash(k), r.grade);
    h = mix(h, r.param_idx);
    h = mix_double(h, r.count);
    h = mix(h, r.control_behavior);
    h = mix(h, r.max_queueing_time_ms);
    h = mix(h, r.burst_count);
    const uint64_t d = (uint64_t)r.duration_in_sec;
    h = mix(h, (int32_t)(uint32_t)(d ^ (d >> 32)));
    h = mix(h, k.extra_hash);
    h = mix(h, 0);
    return mix(h, 0);
}
bool flow_equal(const sf_flow_rule& a, const sf_rule_key& ka, const sf_flow_rule& b, const sf_rule_key& kb) {
    return a.resource == b.resource && ka.limit_app_id == kb.limit_app_id && a.grade == b.grade &&
           same_double(a.count, b.count) && a.strategy == b.strategy && a.control_behavior == b.control_behavior &&
           a.warm_up_period_sec == b.warm_up_period_sec && a.max_queueing_time_ms == b.max_queueing_time_ms &&
           (a.cluster_mode != 0) == (b.cluster_mode != 0) && a.ref_resource == b.ref_resource &&
           ka.extra_hash == kb.extra_hash && ka.cluster_hash == kb.cluster_hash;
}
// FlowRuleComparator.compare (:30-55): cluster-mode rules last, "default" after specific origins
int flow_compare(const sf_flow_rule& a, const sf_rule_key& ka, const sf_flow_rule& b, const sf_rule_key& kb) {
    if (a.cluster_mode && !b.cluster_mode) return 1;
    if (!a.cluster_mode && b.cluster_mode) return -1;
    if (ka.limit_app_id == kb.limit_app_id) return 0;
    if (ka.limit_app_id == 0) return 1;
    if (kb.limit_app_id == 0) return -1;
    return 0;
}

uint32_t spread(int32_t h, uint32_t cap) {                     // HashMap.hash + index
    const uint32_t x = (uint32_t)h;
    return (x ^ (x >> 16)) & (cap - 1);
}

// HashSet iteration order of elements added in turn with these hashes (JDK 8
// HashMap: table 16, doubles past 0.75 load; a bin reaching 9 entries in a
// table under 64 doubles it; entries of a bin in insertion order).  false:
// a bin would be treeified (not modelled).
bool hashset_order(const std::vector<int32_t>& h, std::vector<uint32_t>& order) {
    uint32_t cap = 16;
    for (size_t k = 0; k < h.size(); k++) {
        for (;;) {
            uint32_t same = 0;
            const uint32_t b = spread(h[k], cap);
            for (size_t j = 0; j <= k; j++) same += spread(h[j], cap) == b;
            if (same < 9) break;
            if (cap >= 64) return false;
            cap *= 2;
        }
        if (k + 1 > (size_t)(cap * 3 / 4)) cap *= 2;
    }
    order.resize(h.size());
    for (uint32_t k = 0; k < order.size(); k++) order[k] = k;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return spread(h[a], cap) < spread(h[b], cap); });
    return true;
}

template <class R, class Valid, class Hash, class Eq, class Cmp>
int rule_order(const R* rules, const sf_rule_key* keys, uint32_t n, uint32_t* out, uint32_t* n_out, Valid valid,
               Hash hash, Eq eq, Cmp cmp) {
    std::map<uint32_t, std::vector<uint32_t>> by_res;          // resource -> kept rules (insertion order)
    std::vector<uint32_t> first_seen;
    for (uint32_t i = 0; i < n; i++) {
        if (!valid(rules[i])) continue;
        auto it = by_res.find(rules[i].resource);
        if (it == by_res.end()) { first_seen.push_back(rules[i].resource); it = by_res.emplace(rules[i].resource, std::vector<uint32_t>{}).first; }
        bool dup = false;
        for (uint32_t j : it->second) if (eq(rules[j], keys[j], rules[i], keys[i])) { dup = true; break; }
        if (!dup) it->second.push_back(i);
    }
    uint32_t m = 0;
    for (uint32_t res : first_seen) {
        const std::vector<uint32_t>& kept = by_res[res];
        std::vector<int32_t> hs(kept.size());
        for (size_t k = 0; k < kept.size(); k++) hs[k] = hash(rules[kept[k]], keys[kept[k]]);
        std::vector<uint32_t> ord;
        if (!hashset_order(hs, ord)) return SF_ERR_UNSUPPORTED;
        std::vector<uint32_t> lst(ord.size());
        for (size_t k = 0; k < ord.size(); k++) lst[k] = kept[ord[k]];
        std::stable_sort(lst.begin(), lst.end(),
                         [&](uint32_t a, uint32_t b) { return cmp(rules[a], keys[a], rules[b], keys[b]) < 0; });
        for (uint32_t x : lst) out[m++] = x;
    }
    *n_out = m;
    return SF_OK;
}

}  // namespace

extern "C" {

int sf_flow_rule_order(const sf_flow_rule* rules, const sf_rule_key* keys, uint32_t n, uint32_t* order,
                       uint32_t* n_out) {
    if ((n && (!rules || !keys || !order)) || !n_out) return SF_ERR_INVALID;
    return rule_order(rules, keys, n, order, n_out, [](const sf_flow_rule& r) { return valid_flow_rule(r); },
                      flow_hash, flow_equal, flow_compare);
}

int sf_param_rule_order(const sf_param_rule* rules, const sf_rule_key* keys, uint32_t n, const sf_hot_item* items,
                        uint32_t n_items, uint32_t* order, uint32_t* n_out) {
    if ((n && (!rules || !keys || !order)) || !n_out || (n_items && !items)) return SF_ERR_INVALID;
    for (uint32_t i = 0; i < n; i++)
        if ((uint64_t)rules[i].item_offset + rules[i].item_count > n_items) return SF_ERR_INVALID;
    auto eq = [&](const sf_param_rule& a, const sf_rule_key& ka, const sf_param_rule& b, const sf_rule_key& kb) {
        if (!(a.resource == b.resource && ka.limit_app_id == kb.limit_app_id && a.grade == b.grade &&
              a.param_idx == b.param_idx && same_double(a.count, b.count) && a.control_behavior == b.control_behavior &&
              a.max_queueing_time_ms == b.max_queueing_time_ms && a.burst_count == b.burst_count &&
              a.duration_in_sec == b.duration_in_sec && a.item_count == b.item_count && ka.extra_hash == kb.extra_hash))
            return false;
        for (uint32_t t = 0; t < a.item_count; t++) {
            const sf_hot_item &x = items[a.item_offset + t], &y = items[b.item_offset + t];
            if (x.tag != y.tag || x.bits != y.bits || x.count != y.count) return false;
        }
        return true;
    };
    // ParamFlowRuleUtil.isValidRule (ParamFlowRuleUtil.java:46-52); local rules (checkCluster: true)
    auto valid = [](const sf_param_rule& r) {
        return r.count >= 0 && r.grade >= 0 && r.burst_count >= 0 && r.control_behavior >= 0 &&
               r.duration_in_sec > 0 && r.max_queueing_time_ms >= 0;
    };
    auto unsorted = [](const sf_param_rule&, const sf_rule_key&, const sf_param_rule&, const sf_rule_key&) { return 0; };
    return rule_order(rules, keys, n, order, n_out, valid, param_hash, eq, unsorted);
}

}  // extern "C"
