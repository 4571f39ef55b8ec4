// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 16, 18, 20, 22.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(16)
GOL_RESIDENT_RW(18)
GOL_RESIDENT_RW(20)
GOL_RESIDENT_RW(22)
