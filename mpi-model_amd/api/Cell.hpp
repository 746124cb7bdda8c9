// Cell.hpp -- a cell of the rectangular space (reference: src/Cell.hpp:9-158).
// SetNeighbor() classifies the cell against the GLOBAL grid DIMX x DIMY exactly as the
// reference does (corner 3, edge 5, interior 8 Moore neighbours, Cell.hpp:71-157) and
// lists the neighbour coordinates (x in neighbors[0..7], y in neighbors[8..15]).
// Differences, both fixes: copies keep all 16 coordinates (the reference copies 8,
// Cell.hpp:33-34,45-46), and the (DIMX-1, 0) corner lists its real neighbours (the
// reference lists (x-1, y-1), Cell.hpp:102). On the device no Cell exists: coordinates
// and neighbour counts are derived from the cell index.
#ifndef CELL_HPP
#define CELL_HPP

#include "Attribute.hpp"
#include "Defines.hpp"

template <typename T>
class Cell {
public:
    int x;
    int y;
    Attribute<T> attribute;
    int neighbors[NEIGHBORS + NEIGHBORS];
    int count_neighbors;

    Cell() : x(0), y(0), count_neighbors(0) { clear_neighbors(); }
    Cell(const int& x_, const int& y_, const Attribute<T>& a)
        : x(x_), y(y_), attribute(a), count_neighbors(0) {
        clear_neighbors();
    }
    Cell(const Cell<T>& o) { *this = o; }
    ~Cell() {}
    Cell<T>& operator=(const Cell<T>& o) {
        x = o.x;
        y = o.y;
        attribute = o.attribute;
        count_neighbors = o.count_neighbors;
        for (int i = 0; i < NEIGHBORS + NEIGHBORS; ++i) neighbors[i] = o.neighbors[i];
        return *this;
    }

    void SetX(const int& v) { x = v; }
    void SetY(const int& v) { y = v; }
    void SetAttribute(const Attribute<T>& a) { attribute = a; }
    int GetX() { return x; }
    int GetY() { return y; }
    Attribute<T> GetAttribute() { return attribute; }

    // A copy of this cell with its Moore neighbourhood inside DIMX x DIMY filled in.
    Cell<T> SetNeighbor() const {
        Cell<T> c = *this;
        c.count_neighbors = 0;
        for (int dx = -1; dx <= 1; ++dx)
            for (int dy = -1; dy <= 1; ++dy) {
                const int nx = x + dx, ny = y + dy;
                if ((dx == 0 && dy == 0) || nx < 0 || ny < 0 || nx >= DIMX || ny >= DIMY) continue;
                c.neighbors[c.count_neighbors] = nx;
                c.neighbors[NEIGHBORS + c.count_neighbors] = ny;
                ++c.count_neighbors;
            }
        return c;
    }

private:
    void clear_neighbors() {
        for (int i = 0; i < NEIGHBORS + NEIGHBORS; ++i) neighbors[i] = 0;
    }
};

#endif
