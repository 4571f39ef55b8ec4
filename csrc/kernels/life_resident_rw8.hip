// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 80, 88.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(80)
GOL_RESIDENT_RW(88)
