// Test infrastructure: the AlphaZero root-noise vectors exactly as the reference draws them
// (lzero/mcts/ctree/ctree_alphazero/mcts_alphazero.cpp:58-81): a default-seeded
// std::default_random_engine and std::gamma_distribution<double>(alpha, 1) per call, normalised —
// so the vector only depends on (alpha, number of children). Built with g++/libstdc++ like the
// reference. out[(n - 1) * max_n + i] = i-th noise of a node with n children, n = 1..max_n.
#include <random>
#include <vector>

extern "C" void lzo_az_noise_table(double alpha, int max_n, double *out) {
  for (int n = 1; n <= max_n; ++n) {
    std::default_random_engine generator;
    std::gamma_distribution<double> distribution(alpha, 1.0);
    std::vector<double> noise;
    double sum = 0;
    for (int i = 0; i < n; ++i) {
      double s = distribution(generator);
      noise.push_back(s);
      sum += s;
    }
    for (int i = 0; i < max_n; ++i) out[(n - 1) * max_n + i] = i < n ? noise[i] / sum : 0.0;
  }
}
