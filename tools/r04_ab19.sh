# round 4: scheduling constants re-checked after the argument laundering: S0 HEAD (tester class at >= 1/3 of the live lanes,
# AppendEntries deferral while >= 32 other node events) | T14 tester 1/4 | T25 tester 2/5 | AO24 / AO40 deferral floor 24 / 40
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or snapshot_install_unreliable_2d)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash snapshot_install_unreliable_2d" bash tools/ab.sh ab19 S0 T14 T25 AO24 AO40 || exit 1
