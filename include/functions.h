/* functions.h — drop-in for parallel-implementation/functions.h:1-12, the objective header the
 * CUDA path's callers include (L-BFGS.cu:12 and the four variants). Same four declarations; the
 * definitions are this library's (functions.cpp:6-49 formulas, = benchmark.cpp:58-81 and
 * main.cpp:7-21), and passed to LBFGS_CUDA() (lbfgs.h) they run on the GPU. */
#ifndef LBFGS_AMD_FUNCTIONS_H
#define LBFGS_AMD_FUNCTIONS_H
#include <iostream>
#include <vector>

#include "lbfgs.h"

using namespace std;  // as the reference header (functions.h:4); its callers rely on it

double quadratic(const vector<double>& X);
vector<double> quadratic_grad(const vector<double>& X);
double rosenbrock(const vector<double>& X);
vector<double> rosenbrock_grad(const vector<double>& X);

#endif
