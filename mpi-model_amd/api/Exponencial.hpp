// Exponencial.hpp -- exponential outflow: rate x value (reference: src/Exponencial.hpp:7-21).
// execute() uses the flow's captured copy of the source value (Exponencial.hpp:15);
// execute(cell) is the per-cell form (Exponencial.hpp:18-20) that the GPU step applies
// to every cell of a whole-grid flow.
#ifndef EXPONENCIAL_HPP
#define EXPONENCIAL_HPP

#include "Flow.hpp"

template <class T>
class Exponencial : public Flow<T> {
public:
    Exponencial() : Flow<T>() {}
    Exponencial(const Cell<T>& cell, const double& rate) : Flow<T>(cell, rate) {}
    explicit Exponencial(const double& rate) : Flow<T>(rate) {}

    double execute() { return this->flow_rate * this->source.attribute.value; }
    double execute(const Cell<T>& cell) { return this->flow_rate * cell.attribute.value; }
};

#endif
