// Flow.hpp -- a flow of attribute value out of a source (reference: src/Flow.hpp:7-58).
// Reference form: Flow(source_cell, rate) -- one source cell whose value the flow
// captures at construction (Flow.hpp:19); Model applies it once (src/Model.hpp:176-235).
// Extension: Flow(rate) -- every cell of the space is a source, every step
// (the generalisation BASELINE.json names); `attribute` selects the attribute.
#ifndef FLOW_HPP
#define FLOW_HPP

#include "Cell.hpp"

template <class T>
class Flow {
public:
    Cell<T> source;
    int target[NEIGHBORS + NEIGHBORS];
    int count_targets;
    double flow_rate;
    double last_execute;
    bool whole_grid;  // extension: every cell emits (Flow(rate))
    int attribute;    // extension: attribute index the flow moves

    Flow() : count_targets(0), flow_rate(0.0), last_execute(0.0), whole_grid(false), attribute(0) {
        for (int i = 0; i < NEIGHBORS + NEIGHBORS; ++i) target[i] = 0;
    }
    Flow(const Cell<T>& cell, const double& rate)
        : source(cell), count_targets(cell.count_neighbors), flow_rate(rate), last_execute(0.0),
          whole_grid(false), attribute(0) {
        for (int i = 0; i < NEIGHBORS + NEIGHBORS; ++i) target[i] = cell.neighbors[i];
    }
    explicit Flow(const double& rate)
        : count_targets(0), flow_rate(rate), last_execute(0.0), whole_grid(true), attribute(0) {
        for (int i = 0; i < NEIGHBORS + NEIGHBORS; ++i) target[i] = 0;
    }
    Flow(const Flow<T>& o) { *this = o; }
    Flow<T>& operator=(const Flow<T>& o) {
        source = o.source;
        count_targets = o.count_targets;
        for (int i = 0; i < NEIGHBORS + NEIGHBORS; ++i) target[i] = o.target[i];
        flow_rate = o.flow_rate;
        last_execute = o.last_execute;
        whole_grid = o.whole_grid;
        attribute = o.attribute;
        return *this;
    }
    virtual ~Flow() {}

    virtual double execute() = 0;
};

#endif
