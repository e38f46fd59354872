// Internal interfaces of the host runtime shared by its translation units (ctok_host.cpp defines
// them; trainer_host.cpp uses them).  Not part of the C ABI.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

struct ctok;

namespace ctok_host {
// Throw a CTOK_E_* error (message for ctok_last_error); run_guarded turns it into the return code.
[[noreturn]] void throw_error(int code, const std::string& msg);
int run_guarded(const std::function<void()>& f);
// GPU pre-tokenization of a host batch with tokenizer t on device dev: the text the pieces index
// (NFC-normalised when normalisation ran), its doc offsets and the piece-start bitmap.
void pretokenize(ctok* t, int dev, const uint8_t* utf8, const uint64_t* doc_off, uint64_t n_docs,
                 std::vector<uint8_t>& text, std::vector<uint64_t>& off, std::vector<uint32_t>& pbits);
// CPUs this process may run on: the affinity mask, capped by the cgroup v2 CPU quota (cpu.max) --
// what Rust's available_parallelism (rayon's default pool size) reports on Linux; >= 1
unsigned usable_cpus();
}  // namespace ctok_host
