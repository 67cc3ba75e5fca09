// SPDX-License-Identifier: LGPL-2.1
//
// dmclock_recs.h / dmclock_util.h equivalents for the MI355X engine's C++
// facade: the value types the reference's callers use
// (/root/reference/src/dmclock_recs.h:25-72, dmclock_util.h:33-52).
#pragma once

#include <cassert>
#include <cmath>
#include <cstdint>
#include <ctime>
#include <limits>
#include <ostream>

namespace crimson {
namespace dmclock {

using Counter = uint64_t;  // dmclock_recs.h:25
using Cost = uint32_t;     // dmclock_recs.h:31

enum class PhaseType : uint8_t { reservation, priority };  // dmclock_recs.h:33

inline std::ostream& operator<<(std::ostream& out, const PhaseType& phase) {
  return out << (phase == PhaseType::reservation ? "reservation" : "priority");
}

// dmclock_recs.h:40-72
struct ReqParams {
  uint32_t delta;  // count of all replies since last request
  uint32_t rho;    // count of reservation replies since last request
  ReqParams(uint32_t d, uint32_t r) : delta(d), rho(r) { assert(rho <= delta); }
  ReqParams() : ReqParams(0, 0) {}
  ReqParams(const ReqParams& o) = default;
  friend std::ostream& operator<<(std::ostream& out, const ReqParams& rp) {
    return out << "ReqParams{ delta:" << rp.delta << ", rho:" << rp.rho << " }";
  }
};

// dmclock_util.h:33-52: Time is seconds since the epoch as a double
using Time = double;
static const Time TimeZero = 0.0;
static const Time TimeMax = std::numeric_limits<Time>::max();

inline Time get_time() {
  struct timespec now;
  clock_gettime(CLOCK_REALTIME, &now);
  return now.tv_sec + (now.tv_nsec / 1.0e9);
}

}  // namespace dmclock
}  // namespace crimson
