/* line_search.h — drop-in for sequential-implementation/line_search.h:1-27 (signatures) and the
 * interpolation helpers of line_search.cpp:8-16. Each search runs the same logic as inside
 * LBFGS() with every trial evaluated on the GPU (lbfgs_line_search): objectives from
 * benchmark.h on the device, any other callable through host callbacks at the trial points.
 * Returns the step size alpha like the reference. */
#ifndef LINE_SEARCH_H
#define LINE_SEARCH_H

#include <functional>
#include <vector>

using namespace std;  // as the reference header (line_search.h:7)

double cubicInterpolate(double alpha0, double alpha1, double phi0, double dphi0, double phi1, double dphi1);
double quadraticInterpolate(double alpha0, double alpha1, double phi0, double dphi0, double phi1);

double backtrackingLineSearch(const vector<double>& x, const vector<double>& d,
                              const function<double(vector<double>)>& f,
                              const vector<double>& gradient);

double backtrackingWolfeLineSearch(const vector<double>& x, const vector<double>& d,
                                   const function<double(vector<double>)>& f,
                                   const function<vector<double>(vector<double>)>& grad,
                                   const vector<double>& gradient);

double armijoInterpolationLineSearch(const vector<double>& x, const vector<double>& d,
                                     const function<double(vector<double>)>& f,
                                     const vector<double>& gradient);

double wolfeInterpolationLineSearch(const vector<double>& x, const vector<double>& d,
                                    const function<double(vector<double>)>& f,
                                    const function<vector<double>(vector<double>)>& grad,
                                    const vector<double>& gradient);

#endif  // LINE_SEARCH_H
