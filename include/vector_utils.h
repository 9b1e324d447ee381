/* vector_utils.h — drop-in for sequential-implementation/vector_utils.h:1-30 (same names and
 * signatures; parallel-implementation/vector_utils.h:1-16 is a subset). The BLAS-1 functions run
 * on the GPU through the C ABI (lbfgs_dev_dot / lbfgs_dev_elementwise) with the canonical
 * reduction order; printing and averaging stay host helpers as in the reference. */
#ifndef VECTOR_UTILS_H
#define VECTOR_UTILS_H

#include <cmath>
#include <iostream>
#include <vector>

using namespace std;  // as the reference header (vector_utils.h:8); callers rely on it

void printMatrix(const vector<vector<double>> &matrix);
void printVector(const vector<double> &vector);
void ensureSameSize(const vector<double> &v1, const vector<double> &v2);  // throws logic_error
double dotProduct(const vector<double> &v1, const vector<double> &v2);
vector<double> scalarProduct(const double scalar, const vector<double> &v);
vector<double> add(const vector<double> &v1, const vector<double> &v2);
vector<double> negative(const vector<double> &v);
double vectorNorm(const vector<double> &v);
double getRho(const vector<double> &s, const vector<double> &y);
double calculateAverage(std::vector<double> &values);

#endif
