// MPIImpl.cpp -- blocking typed send/receive on MPI_COMM_WORLD; failures throw
// std::runtime_error (reference: src/MPIImpl.cpp:6-15).
#include "MPIImpl.hpp"

#include <stdexcept>

void SendImpl(void* data, int count, Abstraction::DataType type, int dest, int tag) {
    const int rc = MPI_Send(data, count, ConvertType(type), dest, tag, MPI_COMM_WORLD);
    if (rc != MPI_SUCCESS) throw std::runtime_error("MPI_Send failed");
}

void ReceiveImpl(void* data, int count, Abstraction::DataType type, int src, int tag) {
    MPI_Status status;
    const int rc = MPI_Recv(data, count, ConvertType(type), src, tag, MPI_COMM_WORLD, &status);
    if (rc != MPI_SUCCESS) throw std::runtime_error("MPI_Recv failed");
}
