// walk.h -- internal: the install walk (walk.cpp, host-only).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "reflow_hip.h"

// internal/walker Scan order and os.Stat semantics; rel / full paths and
// Stat sizes of every non-directory entry.
int walk_tree(const char* root, std::vector<std::string>& rel, std::vector<std::string>& full,
              std::vector<int64_t>& sizes);
