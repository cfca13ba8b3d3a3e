// walk.cpp -- internal/walker's Scan (walker.go:33-99) as Executor.install
// uses it (local/executor.go:514-557), host-only: the listing rf_install_dir
// digests, also exported alone (rf_walk_*).
//   * os.Stat semantics: symlinks are followed; ENOENT (e.g. a dangling link)
//     skips the entry (walker.go:40-43); any other stat/readdir error fails.
//   * directory entries sorted bytewise (readDirNames, walker.go:88-99),
//     depth-first pre-order (children prepended to the todo list, :52-55).
//   * relpath = filepath.Rel(root, path): "." for a root that is a file.
//   * Size = the Stat size (executor.go:525 takes w.Info().Size()).
// Regular files' sizes come from a parallel stat pass (<= 60 threads, the
// DigestLimiter of local/executor.go:41).  No HIP: builds into the sanitizer
// test (make asan).
#include <dirent.h>
#include <errno.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "errors.h"
#include "walk.h"

using rf::fail;

namespace {
struct Entries {
    std::vector<std::string>& rel;
    std::vector<std::string>& full;
    std::vector<int64_t>& sizes;
};
}  // namespace

// Entry `path` (stat follows links, as os.Stat).  A directory is read,
// sorted and closed before its children are visited, so the walk holds one
// directory open at a time whatever the depth (walker.Scan closes each
// directory after Readdirnames too).
static int walk_rec(const std::string& path, const std::string& rel, Entries& in, int depth) {
    struct stat st;
    if (::stat(path.c_str(), &st) != 0) {
        if (errno == ENOENT) return RF_OK;
        return fail(RF_EIO, "stat %s: %s", path.c_str(), strerror(errno));
    }
    if (!S_ISDIR(st.st_mode)) {
        in.full.push_back(path);
        in.rel.push_back(rel);
        in.sizes.push_back((int64_t)st.st_size);
        return RF_OK;
    }
    if (depth > 4096) return fail(RF_EIO, "walk %s: directory nesting deeper than 4096 (link cycle?)", path.c_str());
    DIR* d = ::opendir(path.c_str());
    if (!d) return fail(RF_EIO, "open %s: %s", path.c_str(), strerror(errno));
    std::vector<std::pair<std::string, unsigned char>> names;
    errno = 0;
    while (struct dirent* de = ::readdir(d)) {
        if (strcmp(de->d_name, ".") && strcmp(de->d_name, "..")) names.emplace_back(de->d_name, de->d_type);
        errno = 0;
    }
    const int rerr = errno;
    ::closedir(d);
    if (rerr) return fail(RF_EIO, "readdir %s: %s", path.c_str(), strerror(rerr));
    // char_traits<char>: bytewise (unsigned) order
    std::sort(names.begin(), names.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (const auto& [nm, type] : names) {
        std::string cpath = path + "/" + nm, crel = rel == "." ? nm : rel + "/" + nm;
        if (type == DT_REG) {
            // a regular file (not a link): its Stat size is taken by the
            // parallel pass below (-1 = pending)
            in.full.push_back(std::move(cpath));
            in.rel.push_back(std::move(crel));
            in.sizes.push_back(-1);
        } else if (int rc = walk_rec(cpath, crel, in, depth + 1)) {  // dirs, links, unknown: stat
            return rc;
        }
    }
    return RF_OK;
}

int walk_tree(const char* root, std::vector<std::string>& rel, std::vector<std::string>& full,
              std::vector<int64_t>& sizes) {
    ARG(root, "null root");
    Entries in{rel, full, sizes};
    int rc = walk_rec(root, ".", in, 0);
    if (rc) return rc;
    {
        // Stat sizes of the regular files the walk did not stat, in parallel;
        // one removed since the readdir is skipped, as the walker's Stat would
        std::vector<uint64_t> pend;
        for (uint64_t i = 0; i < in.sizes.size(); ++i)
            if (in.sizes[i] < 0) pend.push_back(i);
        std::vector<int> err(pend.size(), 0);
        std::atomic<uint64_t> nx{0};
        auto st_worker = [&]() {
            for (uint64_t k; (k = nx.fetch_add(1)) < pend.size();) {
                struct stat st;
                if (::stat(in.full[pend[k]].c_str(), &st) == 0)
                    in.sizes[pend[k]] = (int64_t)st.st_size;
                else
                    err[k] = errno;
            }
        };
        const uint64_t hw = std::max(1u, std::thread::hardware_concurrency());
        const uint64_t nt = std::min<uint64_t>({60, hw, pend.size() / 64 + 1});
        std::vector<std::thread> pool;
        for (uint64_t t = 1; t < nt; ++t) pool.emplace_back(st_worker);
        st_worker();
        for (auto& t : pool) t.join();
        bool drop = false;
        for (uint64_t k = 0; k < pend.size(); ++k) {
            if (err[k] == ENOENT) {
                drop = true;
            } else if (err[k]) {
                return fail(RF_EIO, "stat %s: %s", in.full[pend[k]].c_str(), strerror(err[k]));
            }
        }
        if (drop) {  // rare: compact out the vanished entries (sizes still -1)
            uint64_t w = 0;
            for (uint64_t i = 0; i < in.sizes.size(); ++i) {
                if (in.sizes[i] < 0) continue;
                in.full[w] = std::move(in.full[i]);
                in.rel[w] = std::move(in.rel[i]);
                in.sizes[w++] = in.sizes[i];
            }
            in.full.resize(w);
            in.rel.resize(w);
            in.sizes.resize(w);
        }
    }
    return RF_OK;
}

struct rf_walk {
    std::vector<std::string> rel, full;
    std::vector<int64_t> sizes;
};

extern "C" int rf_walk_dir(const char* root, rf_walk** out) {
    ARG(root && out, "null argument");
    *out = nullptr;
    auto* w = new rf_walk();
    int rc = walk_tree(root, w->rel, w->full, w->sizes);
    if (rc) {
        delete w;
        return rc;
    }
    *out = w;
    return RF_OK;
}

extern "C" int rf_walk_info(const rf_walk* w, uint64_t* n_entries, uint64_t* path_bytes) {
    ARG(w && n_entries && path_bytes, "null argument");
    uint64_t b = 0;
    for (const auto& r : w->rel) b += r.size();
    *n_entries = w->rel.size();
    *path_bytes = b;
    return RF_OK;
}

extern "C" int rf_walk_entries(const rf_walk* w, char* paths, uint64_t* path_offs, int64_t* sizes) {
    ARG(w && path_offs && (w->rel.empty() || sizes), "null argument");
    uint64_t o = 0;
    for (size_t i = 0; i < w->rel.size(); ++i) {
        path_offs[i] = o;
        if (paths && !w->rel[i].empty()) memcpy(paths + o, w->rel[i].data(), w->rel[i].size());
        o += w->rel[i].size();
        sizes[i] = w->sizes[i];
    }
    path_offs[w->rel.size()] = o;
    return RF_OK;
}

extern "C" void rf_walk_free(rf_walk* w) { delete w; }
