// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 24, 26, 28, 30.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(24)
GOL_RESIDENT_RW(26)
GOL_RESIDENT_RW(28)
GOL_RESIDENT_RW(30)
