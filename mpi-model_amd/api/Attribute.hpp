// Attribute.hpp -- the simulated quantity of a cell: {key, value}
// (reference: src/Attribute.hpp:6-46). On the device the engine keeps one fp64
// array per attribute (structure of arrays); this class is the host-side value.
#ifndef ATTRIBUTE_HPP
#define ATTRIBUTE_HPP

template <typename T>
class Attribute {
public:
    int key;
    T value;

    Attribute() : key(0), value() {}
    Attribute(const int& key_, const T& value_) : key(key_), value(value_) {}
    Attribute(const Attribute<T>& o) : key(o.key), value(o.value) {}
    ~Attribute() {}
    Attribute<T>& operator=(const Attribute<T>& o) {
        key = o.key;
        value = o.value;
        return *this;
    }

    int GetKey(void) { return key; }
    void SetKey(const int& k) { key = k; }
    T GetValue(void) { return value; }
    void SetValue(const T& v) { value = v; }
};

#endif
