// Internal helpers shared by the host pre-pass and the device path.
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <memory>
#include <vector>

#include "weightedld.h"

namespace wld {

// Thread-local message behind wld_last_error().
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

// Returns status after recording a message.
int fail(int status, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// std::allocator that leaves trivially constructible elements uninitialised on
// resize: buffers that are written in full right after sizing skip a serial
// zero fill and get their first touch in the threads that write them.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
    template <class U>
    void construct(U *p) noexcept {
        ::new ((void *)p) U;
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new ((void *)p) U(std::forward<A>(a)...);
    }
};

// lib.rs:158-173 — SiteSet: site-major symbols, optional site_map, histograms.
struct SiteSet {
    size_t n_sites = 0;
    size_t n_seqs = 0;
    std::vector<uint8_t, NoInitAlloc<uint8_t>> buffer;  // buffer[site * n_seqs + seq] (resize leaves it unset)
    bool has_map = false;
    std::vector<uint64_t> site_map;   // filtered -> parent index (lib.rs:165-169)
    std::vector<uint64_t> hist;       // 6 per site (lib.rs:171-172)
};

void histogram(const uint8_t *sym, size_t n, uint64_t out[6]);
void major_minor(const uint64_t h[6], int *maj, int *mnr);
void compute_histograms(SiteSet &s);

}  // namespace wld

struct wld_siteset {
    wld::SiteSet s;
};
