bash tools/ab_libs.sh "" c0 c1w3 && bash tools/pmc6.sh v6c1 ""
