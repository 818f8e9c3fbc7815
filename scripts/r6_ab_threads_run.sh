# The r6aa variants of scripts/r6_ab_threads.sh.
export VARIANTS='base|l3|{};b8|l3|{"bindWorkers":8};b4|l3|{"bindWorkers":4};x2|l3x2|{}'
TAG=${TAG:-r6aa} bash scripts/r6_ab_threads.sh
