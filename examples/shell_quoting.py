# Quotes, dollar signs and backslashes reach the interpreter untouched
# (sources are written to a file and run by python, no shell in between).
print("single 'quoted' text")
print('double "quoted" text')
print("literal $HOME and ${PATH}")
print("back\\slash")
