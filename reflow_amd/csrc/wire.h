// wire.h -- internal: host-only wire formats (wire.cpp): Fileset JSON and the
// liveset bloom filter's binary / JSON forms.  No HIP; the sanitizer build
// (make asan) links these units alone.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "reflow_hip.h"

int fileset_check_tree(const rf_fileset_tree* t);
// json.Marshal(node root) appended to o
int fileset_marshal_append(const rf_fileset_tree* t, uint32_t root, std::string& o);
// bloom.ReadFrom / UnmarshalJSON: m, k, the bitset length and its
// wordsNeeded(length) words
int bloom_parse_binary(const uint8_t* buf, size_t len, uint64_t* m, uint64_t* k, uint64_t* length,
                       std::vector<uint64_t>& words);
int bloom_parse_json(const char* json, size_t len, uint64_t* m, uint64_t* k, uint64_t* length,
                     std::vector<uint64_t>& words);
