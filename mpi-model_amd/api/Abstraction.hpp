// Abstraction.hpp -- intrinsic-type tags for the typed message helpers
// (reference: src/Abstraction.hpp:7-76). Unsupported types throw, as there.
#ifndef ABSTRACTION_HPP
#define ABSTRACTION_HPP

#include <stdexcept>

namespace Abstraction {
typedef enum {
    type_unknown = 0,
    type_char,
    type_unsigned_char,
    type_short,
    type_unsigned_short,
    type_int,
    type_unsigned_int,
    type_long,
    type_unsigned_long,
    type_float,
    type_double
} DataType;
}

template <class T>
Abstraction::DataType getAbstractionDataType() {
    throw std::runtime_error("Intrinsic type not supported by the abstraction.");
}

#define MM_ABSTRACTION_TAG(T, TAG) \
    template <>                    \
    inline Abstraction::DataType getAbstractionDataType<T>() { return Abstraction::TAG; }
MM_ABSTRACTION_TAG(char, type_char)
MM_ABSTRACTION_TAG(unsigned char, type_unsigned_char)
MM_ABSTRACTION_TAG(short, type_short)
MM_ABSTRACTION_TAG(unsigned short, type_unsigned_short)
MM_ABSTRACTION_TAG(int, type_int)
MM_ABSTRACTION_TAG(unsigned int, type_unsigned_int)
MM_ABSTRACTION_TAG(long, type_long)
MM_ABSTRACTION_TAG(unsigned long, type_unsigned_long)
MM_ABSTRACTION_TAG(float, type_float)
MM_ABSTRACTION_TAG(double, type_double)
#undef MM_ABSTRACTION_TAG

#endif
