"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, %."""
import csv
import sys

for p in sys.argv[1:]:
    print("==", p)
    for x in csv.DictReader(open(p)):
        print("%-70s %5s %10.1f us %6.2f%%" % (x["Name"][:70], x["Calls"], float(x["AverageNs"]) / 1e3,
                                             float(x["Percentage"])))
