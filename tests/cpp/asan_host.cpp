// asan_host.cpp -- the host-only C-ABI code under AddressSanitizer and
// UndefinedBehaviorSanitizer (reflow_amd/csrc/Makefile `asan`; no GPU):
//   * Fileset JSON (wire.cpp): escapes, invalid UTF-8, nested Lists, short
//     output buffers, random trees;
//   * bloom wire forms (wire.cpp): format -> parse round trips, every
//     truncation of a binary form, corrupted JSON, lengths whose word count
//     would wrap;
//   * rf_graph_split (partition_split.cpp): random DAGs and owners, every
//     piece's arrays walked, malformed descs rejected;
//   * the install walk (walk.cpp: rf_walk_dir) over a real tree with links,
//     a dangling link, empty dirs, a file root and a link cycle;
//   * host SHA-256 (host_sha.cpp) against FIPS 180 vectors;
//   * reflow_host.cpp's host-only helpers (Digest text forms, MarshalJSON).
// Prints PASS; any sanitizer report aborts the process.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "reflow_hip.h"
#include "reflow_host.hpp"

namespace rf {
bool host_sha_available();
void host_sha256(const uint8_t* p, uint64_t len, uint8_t out32[32]);
}  // namespace rf

static int fails = 0;
#define EXPECT(c)                                                      \
    do {                                                               \
        if (!(c)) {                                                    \
            fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #c); \
            ++fails;                                                   \
        }                                                              \
    } while (0)

static std::string hex(const uint8_t* p, size_t n) {
    static const char* H = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) {
        s += H[p[i] >> 4];
        s += H[p[i] & 15];
    }
    return s;
}

// ---- Fileset JSON ------------------------------------------------------------
struct Tree {
    std::vector<uint64_t> list_ptr{0}, entry_ptr{0};
    std::vector<uint32_t> list_child, path_lens;
    std::vector<std::string> path_store;
    std::vector<const char*> paths;
    std::vector<uint8_t> ids;
    std::vector<int64_t> sizes;
    uint32_t node(const std::vector<uint32_t>& kids, const std::vector<std::pair<std::string, int64_t>>& ents) {
        for (uint32_t k : kids) list_child.push_back(k);
        list_ptr.push_back(list_child.size());
        for (auto& e : ents) {
            path_store.push_back(e.first);
            path_lens.push_back((uint32_t)e.first.size());
            for (int i = 0; i < 32; ++i) ids.push_back((uint8_t)(e.second * 7 + i));
            sizes.push_back(e.second);
        }
        entry_ptr.push_back(sizes.size());
        return (uint32_t)list_ptr.size() - 2;
    }
    rf_fileset_tree view() {
        paths.clear();
        for (auto& s : path_store) paths.push_back(s.data());
        rf_fileset_tree t;
        t.n_nodes = list_ptr.size() - 1;
        t.list_ptr = list_ptr.data();
        t.list_child = list_child.empty() ? nullptr : list_child.data();
        t.entry_ptr = entry_ptr.data();
        t.paths = paths.empty() ? nullptr : paths.data();
        t.path_lens = path_lens.empty() ? nullptr : path_lens.data();
        t.ids32 = ids.empty() ? nullptr : ids.data();
        t.sizes = sizes.empty() ? nullptr : sizes.data();
        return t;
    }
};

static std::string marshal(const rf_fileset_tree& t, uint32_t root) {
    uint64_t need = 0;
    int rc = rf_fileset_marshal_json(&t, root, nullptr, 0, &need);
    if (!(rc == RF_OK || (rc == RF_EINVAL && need > 0))) fprintf(stderr, "marshal: %s\n", rf_last_error());
    EXPECT(rc == RF_OK || (rc == RF_EINVAL && need > 0));
    std::vector<uint8_t> buf(need ? need : 1);
    if (need > 1) {  // one byte short must fail and write nothing past cap
        uint64_t n2 = 0;
        EXPECT(rf_fileset_marshal_json(&t, root, buf.data(), need - 1, &n2) == RF_EINVAL && n2 == need);
    }
    EXPECT(rf_fileset_marshal_json(&t, root, buf.data(), need, &need) == RF_OK);
    return std::string(buf.begin(), buf.begin() + need);
}

static void test_fileset_json() {
    Tree tr;
    const uint32_t a = tr.node({}, {{"b.txt", 3}, {"a<&>\"\\\n\x01.txt", 5}, {std::string("bad\xff\xfe", 5), 0}});
    const uint32_t e = tr.node({}, {});
    const uint32_t l = tr.node({a, e, a}, {});
    auto t = tr.view();
    const std::string s = marshal(t, a);
    EXPECT(s.find("\\u003c") != std::string::npos && s.find("\\u0026") != std::string::npos);  // HTML-safe
    EXPECT(s.find("\\ufffd") != std::string::npos);                                           // invalid UTF-8
    EXPECT(s.find("\"a<") == std::string::npos);
    EXPECT(s.find("\"a\\u003c") < s.find("\"b.txt\""));  // keys sorted bytewise
    EXPECT(marshal(t, e) == "{}");
    const std::string ls = marshal(t, l);
    EXPECT(ls.rfind("{\"List\":[", 0) == 0);
    uint64_t n = 0;
    EXPECT(rf_fileset_marshal_json(&t, 99, nullptr, 0, &n) != RF_OK);  // root out of range
    Tree dup;
    const uint32_t dn = dup.node({}, {{"same", 1}, {"same", 2}});
    auto dt = dup.view();
    EXPECT(rf_fileset_marshal_json(&dt, dn, nullptr, 0, &n) == RF_EINVAL && n == 0);  // a map has unique keys
    EXPECT(rf_fileset_marshal_json(nullptr, 0, nullptr, 0, &n) != RF_OK);
    // random trees: random path bytes, shared subtrees
    std::mt19937_64 rng(5);
    for (int it = 0; it < 200; ++it) {
        Tree r;
        std::vector<uint32_t> nodes;
        const int nn = 1 + (int)(rng() % 12);
        for (int i = 0; i < nn; ++i) {
            std::vector<uint32_t> kids;
            if (!nodes.empty() && rng() % 2)
                for (int k = (int)(rng() % 4); k > 0; --k) kids.push_back(nodes[rng() % nodes.size()]);
            std::vector<std::pair<std::string, int64_t>> ents;
            for (int k = (int)(rng() % 4); k > 0; --k) {
                std::string p(rng() % 12, '\0');
                for (auto& c : p) c = (char)(rng() & 0xff);
                p += (char)('0' + k);  // distinct keys within a node (a map)
                ents.push_back({p, (int64_t)(rng() % 1000) - 10});
            }
            nodes.push_back(r.node(kids, ents));
        }
        auto rt = r.view();
        const std::string j = marshal(rt, nodes.back());
        EXPECT(!j.empty() && j.front() == '{' && j.back() == '}');
    }
}

// ---- bloom wire forms ----------------------------------------------------------
static void test_bloom_wire() {
    std::mt19937_64 rng(7);
    for (uint64_t length : {0ull, 1ull, 63ull, 64ull, 65ull, 1000ull, 4096ull}) {
        const uint64_t nw = length / 64 + (length % 64 != 0);
        std::vector<uint64_t> w(nw);
        for (auto& x : w) x = rng();
        for (int form = 0; form < 2; ++form) {
            uint64_t need = 0;
            auto fmt = form ? rf_bloom_format_json : rf_bloom_format_binary;
            EXPECT(fmt(1000, 7, length, w.data(), nw, nullptr, 0, &need) == (need ? RF_EINVAL : RF_OK));
            std::vector<uint8_t> buf(need);
            EXPECT(fmt(1000, 7, length, w.data(), nw, buf.data(), need, &need) == RF_OK);
            uint64_t m = 0, k = 0, len2 = 0, n2 = 0;
            std::vector<uint64_t> w2(nw + 1);
            int rc = form ? rf_bloom_parse_json(reinterpret_cast<const char*>(buf.data()), buf.size(), &m, &k, &len2,
                                                w2.data(), w2.size(), &n2)
                          : rf_bloom_parse_binary(buf.data(), buf.size(), &m, &k, &len2, w2.data(), w2.size(), &n2);
            EXPECT(rc == RF_OK && m == 1000 && k == 7 && len2 == length && n2 == nw);
            EXPECT(std::equal(w.begin(), w.end(), w2.begin()));
            // every truncation parses or fails cleanly
            for (size_t cut = 0; cut < buf.size(); ++cut) {
                std::vector<uint8_t> t(buf.begin(), buf.begin() + cut);
                if (form)
                    (void)rf_bloom_parse_json(reinterpret_cast<const char*>(t.data()), t.size(), &m, &k, &len2,
                                              w2.data(), w2.size(), &n2);
                else
                    EXPECT(rf_bloom_parse_binary(t.data(), t.size(), &m, &k, &len2, w2.data(), w2.size(), &n2) !=
                           RF_OK);
            }
            // corrupted bytes
            for (int c = 0; c < 200 && !buf.empty(); ++c) {
                std::vector<uint8_t> t = buf;
                t[rng() % t.size()] = (uint8_t)rng();
                if (form)
                    (void)rf_bloom_parse_json(reinterpret_cast<const char*>(t.data()), t.size(), &m, &k, &len2,
                                              w2.data(), w2.size(), &n2);
                else
                    (void)rf_bloom_parse_binary(t.data(), t.size(), &m, &k, &len2, w2.data(), w2.size(), &n2);
            }
        }
    }
    // a length whose word count would wrap, and m/k too large for uint64
    uint8_t huge[24] = {0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xf0};
    uint64_t m, k, len2, n2;
    EXPECT(rf_bloom_parse_binary(huge, sizeof huge, &m, &k, &len2, nullptr, 0, &n2) == RF_EINVAL);
    const char* js = "{\"m\":99999999999999999999999,\"k\":1,\"b\":\"\"}";
    EXPECT(rf_bloom_parse_json(js, strlen(js), &m, &k, &len2, nullptr, 0, &n2) == RF_EINVAL);
    const char* jb = "{\"m\":5,\"k\":1,\"b\"";
    EXPECT(rf_bloom_parse_json(jb, strlen(jb), &m, &k, &len2, nullptr, 0, &n2) == RF_EINVAL);
    uint64_t one = 1, need;
    EXPECT(rf_bloom_format_binary(1, 1, 1000, &one, 1, nullptr, 0, &need) == RF_EINVAL);  // too few words
}

// ---- rf_graph_split -------------------------------------------------------------
static void test_graph_split() {
    std::mt19937_64 rng(11);
    for (int it = 0; it < 60; ++it) {
        const uint32_t n_in = 1 + rng() % 20, J = 1 + rng() % 200;
        const int nranks = 1 + (int)(rng() % 5);
        std::vector<uint32_t> out_slot(J), tmpl_len(J), hole_pos, hole_slot;
        std::vector<uint64_t> tmpl_off(J), hole_ptr(J + 1, 0);
        std::vector<int32_t> owner(J);
        std::string blob;
        for (uint32_t j = 0; j < J; ++j) {
            out_slot[j] = n_in + j;
            const uint32_t nh = rng() % 4;
            tmpl_off[j] = blob.size();
            tmpl_len[j] = 34 * nh + 8;
            blob += std::string(tmpl_len[j], 'x');
            while (blob.size() % 16) blob += '\0';
            for (uint32_t h = 0; h < nh; ++h) {
                hole_pos.push_back(34 * h + 2);
                hole_slot.push_back((uint32_t)(rng() % (n_in + j)));  // any earlier slot
            }
            hole_ptr[j + 1] = hole_pos.size();
            owner[j] = (int32_t)(rng() % (nranks + 1)) - 1;
        }
        rf_graph_desc d{J, n_in + J, out_slot.data(), tmpl_off.data(), tmpl_len.data(), hole_ptr.data(),
                        hole_pos.empty() ? nullptr : hole_pos.data(), hole_slot.empty() ? nullptr : hole_slot.data(),
                        reinterpret_cast<const uint8_t*>(blob.data()), blob.size()};
        uint64_t jobs_total = 0, exports = 0, imports = 0;
        for (int r = 0; r < nranks; ++r) {
            rf_graph_piece* pc = nullptr;
            EXPECT(rf_graph_split(&d, nranks, r, owner.data(), &pc) == RF_OK);
            if (!pc) continue;
            rf_graph_desc ld;
            rf_graph_part pt;
            const uint32_t* g = nullptr;
            uint32_t ns = 0;
            EXPECT(rf_graph_piece_desc(pc, &ld) == RF_OK && rf_graph_piece_part(pc, &pt) == RF_OK &&
                   rf_graph_piece_slots(pc, &g, &ns) == RF_OK);
            EXPECT(ns == ld.n_slots);
            uint64_t sum = 0;
            for (uint32_t j = 0; j < ld.n_jobs; ++j) {
                EXPECT(ld.out_slot[j] < ld.n_slots);
                for (uint64_t h = ld.hole_ptr[j]; h < ld.hole_ptr[j + 1]; ++h) sum += ld.hole_slot[h] < ld.n_slots;
                sum += ld.tmpl_off[j] + ld.tmpl_len[j] <= blob.size();
            }
            for (uint32_t s = 0; s < ns; ++s) EXPECT(g[s] < n_in + J);
            for (uint32_t i = 0; i < pt.n_export; ++i) EXPECT(pt.export_slot[i] < ld.n_slots);
            for (uint32_t i = 0; i < pt.n_import; ++i)
                EXPECT(pt.import_slot[i] < ld.n_slots && pt.import_bid[i] < (uint64_t)nranks * pt.max_export);
            jobs_total += ld.n_jobs;
            exports += pt.n_export;
            imports += pt.n_import;
            (void)sum;
            rf_graph_piece_free(pc);
        }
        uint64_t want = 0;
        for (uint32_t j = 0; j < J; ++j) want += owner[j] < 0 ? (uint64_t)nranks : 1;
        EXPECT(jobs_total == want);
        EXPECT(imports == 0 || exports > 0);
    }
    // malformed: owner out of range, out_slot out of range, a slot written twice
    uint32_t os[2] = {1, 1}, tl[2] = {8, 8};
    uint64_t to[2] = {0, 16}, hp[3] = {0, 0, 0};
    int32_t ow[2] = {0, 0};
    uint8_t bl[32] = {0};
    rf_graph_desc d{2, 2, os, to, tl, hp, nullptr, nullptr, bl, 32};
    rf_graph_piece* pc = nullptr;
    EXPECT(rf_graph_split(&d, 1, 0, ow, &pc) == RF_EINVAL && !pc);  // slot 1 written twice
    os[1] = 7;
    EXPECT(rf_graph_split(&d, 1, 0, ow, &pc) == RF_EINVAL);  // out of range
    os[1] = 0;
    ow[1] = 3;
    EXPECT(rf_graph_split(&d, 2, 0, ow, &pc) == RF_EINVAL);  // owner out of range
    EXPECT(rf_graph_split(&d, 2, 2, ow, &pc) == RF_EINVAL);  // rank out of range
}

// ---- install walk ------------------------------------------------------------------
static void put_file(const std::string& p, const std::string& body) {
    FILE* f = fopen(p.c_str(), "wb");
    if (!f) {
        ++fails;
        return;
    }
    fwrite(body.data(), 1, body.size(), f);
    fclose(f);
}

static std::vector<std::pair<std::string, int64_t>> walk(const std::string& root, int* rc_out) {
    rf_walk* w = nullptr;
    std::vector<std::pair<std::string, int64_t>> out;
    *rc_out = rf_walk_dir(root.c_str(), &w);
    if (*rc_out != RF_OK) return out;
    uint64_t n = 0, pb = 0;
    EXPECT(rf_walk_info(w, &n, &pb) == RF_OK);
    std::vector<char> paths(pb + 1);
    std::vector<uint64_t> offs(n + 1);
    std::vector<int64_t> sizes(n + 1);
    EXPECT(rf_walk_entries(w, paths.data(), offs.data(), sizes.data()) == RF_OK);
    for (uint64_t i = 0; i < n; ++i) out.push_back({std::string(&paths[offs[i]], offs[i + 1] - offs[i]), sizes[i]});
    rf_walk_free(w);
    return out;
}

static void test_walk() {
    char tmpl[] = "/tmp/rf_asan_walkXXXXXX";
    const char* d = mkdtemp(tmpl);
    if (!d) {
        ++fails;
        return;
    }
    const std::string r(d);
    mkdir((r + "/a").c_str(), 0755);
    mkdir((r + "/empty").c_str(), 0755);
    put_file(r + "/a/x", "hello");
    put_file(r + "/a/y", "");
    put_file(r + "/b.txt", "abc");
    put_file(r + "/Z", "z");
    put_file(r + "/\xc3\xa9", "accent");
    EXPECT(symlink("a", (r + "/link_dir").c_str()) == 0);
    EXPECT(symlink("b.txt", (r + "/link_file").c_str()) == 0);
    EXPECT(symlink("nowhere", (r + "/dangling").c_str()) == 0);
    int rc = 0;
    auto got = walk(r, &rc);
    const std::vector<std::pair<std::string, int64_t>> want = {
        {"Z", 1}, {"a/x", 5}, {"a/y", 0}, {"b.txt", 3}, {"link_dir/x", 5}, {"link_dir/y", 0}, {"link_file", 3},
        {"\xc3\xa9", 6}};
    EXPECT(rc == RF_OK && got == want);
    auto one = walk(r + "/b.txt", &rc);  // a file root: relpath "."
    EXPECT(rc == RF_OK && one.size() == 1 && one[0].first == "." && one[0].second == 3);
    auto none = walk(r + "/does-not-exist", &rc);  // ENOENT: skipped, as walker.go:40-43
    EXPECT(rc == RF_OK && none.empty());
    mkdir((r + "/cyc").c_str(), 0755);
    EXPECT(symlink(".", (r + "/cyc/loop").c_str()) == 0);  // cyc/loop/loop/... : ELOOP or too deep
    (void)walk(r + "/cyc", &rc);
    EXPECT(rc == RF_EIO);
    std::string cmd = "rm -rf '" + r + "'";
    EXPECT(system(cmd.c_str()) == 0);
}

// ---- host SHA-256 ----------------------------------------------------------------
static void test_host_sha() {
    if (!rf::host_sha_available()) return;
    uint8_t o[32];
    rf::host_sha256(reinterpret_cast<const uint8_t*>("abc"), 3, o);
    EXPECT(hex(o, 32) == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");
    rf::host_sha256(nullptr, 0, o);
    EXPECT(hex(o, 32) == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");
    std::string mil(1000000, 'a');
    rf::host_sha256(reinterpret_cast<const uint8_t*>(mil.data()), mil.size(), o);
    EXPECT(hex(o, 32) == "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0");
    for (size_t n = 0; n < 200; ++n) {  // every padding edge runs clean
        std::string m(n, 'q');
        rf::host_sha256(reinterpret_cast<const uint8_t*>(m.data()), n, o);
    }
}

// ---- reflow_host.cpp host-only helpers -------------------------------------------
static void test_host_mirror() {
    reflow::Digest d;
    for (int i = 0; i < 32; ++i) d.b[i] = (uint8_t)i;
    reflow::Digest p;
    EXPECT(reflow::Digest::Parse(d.String(), &p) && p == d);
    EXPECT(!reflow::Digest::Parse("sha256:zz", &p) && !reflow::Digest::Parse("", &p));
    EXPECT(d.Short() == "sha256:00010203");
    reflow::Fileset fs;
    fs.Map["x<y"] = reflow::File{d, 7};
    reflow::Fileset top;
    top.List = std::vector<reflow::Fileset>{fs, reflow::Fileset{}};
    const std::string j = reflow::MarshalJSON(top);
    EXPECT(j.find("\\u003c") != std::string::npos && j.find("\"List\"") != std::string::npos);
    std::string w;
    top.WriteDigest(w);
    EXPECT(!w.empty() && top.N() == 1);
}

// the lowering's open-addressing map against std::unordered_map: random
// inserts / finds / erases (backward-shift deletion keeps every probe run
// intact), keys crowded into a few home slots as well as spread
static void test_flat_map() {
    struct Crowd {  // 8 home slots for every key: long runs, wrap-around
        size_t operator()(uint64_t k) const { return (size_t)(k & 7) * 0x1000001ull; }
    };
    for (int crowd = 0; crowd < 2; ++crowd) {
        reflow::detail::FlatMap<uint64_t, uint32_t, std::hash<uint64_t>> a;
        reflow::detail::FlatMap<uint64_t, uint32_t, Crowd> b;
        std::unordered_map<uint64_t, uint32_t> ref;
        uint64_t x = 12345;
        for (int op = 0; op < 200000; ++op) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            const uint64_t k = (x >> 33) % (crowd ? 300 : 5000);
            const int what = (int)((x >> 20) % 3);
            auto it = ref.find(k);
            if (what == 0 && it == ref.end()) {
                ref[k] = (uint32_t)op;
                if (crowd) b.insert(k, (uint32_t)op); else a.insert(k, (uint32_t)op);
            } else if (what == 1 && it != ref.end()) {
                ref.erase(it);
                EXPECT(crowd ? b.erase(k) : a.erase(k));
            } else {
                const uint32_t* v = crowd ? b.find(k) : a.find(k);
                EXPECT((v != nullptr) == (it != ref.end()));
                if (v && it != ref.end()) EXPECT(*v == it->second);
            }
        }
        EXPECT((crowd ? b.size() : a.size()) == ref.size());
    }
}

// Canonicalize's walk: a wide root's children walked in groups on host
// threads give the sequential post-order node for node (random DAGs with
// shared subgraphs, map flows and a root that lists some children twice)
static void test_post_order() {
    std::mt19937_64 rng(7);
    for (int trial = 0; trial < 4; ++trial) {
        const size_t n = 20000 + 5000 * trial;
        std::vector<reflow::Flow> nodes(n + 1);
        for (size_t i = 0; i < n; ++i) {
            const size_t lo = i > 400 ? i - 400 : 0;
            const int nd = i ? (int)(rng() % 5) : 0;
            for (int k = 0; k < nd; ++k) nodes[i].Deps.push_back(&nodes[lo + rng() % (i - lo)]);
            if (i && rng() % 17 == 0) nodes[i].MapFlow = &nodes[lo + rng() % (i - lo)];
        }
        reflow::Flow& root = nodes[n];
        const size_t nk = 300 + 700 * (size_t)trial;
        for (size_t k = 0; k < nk; ++k) root.Deps.push_back(&nodes[rng() % n]);
        if (trial & 1) root.MapFlow = &nodes[rng() % n];
        std::vector<reflow::Flow*> seq, par;
        reflow::detail::PtrIndex iseq, ipar;
        reflow::detail::PostOrder(&root, 1, seq, iseq);
        reflow::detail::PostOrder(&root, 4, par, ipar);
        EXPECT(seq == par);
        EXPECT(!seq.empty() && seq.back() == &root && iseq.size() == seq.size() && ipar.size() == par.size());
        for (size_t k = 0; k < par.size(); ++k) EXPECT(ipar.find(par[k]) && *ipar.find(par[k]) == k);
    }
}

int main() {
    test_post_order();
    test_flat_map();
    test_fileset_json();
    test_bloom_wire();
    test_graph_split();
    test_walk();
    test_host_sha();
    test_host_mirror();
    if (fails) {
        fprintf(stderr, "%d failures\n", fails);
        return 1;
    }
    printf("PASS\n");
    return 0;
}
