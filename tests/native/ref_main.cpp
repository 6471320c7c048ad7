// The reference's main() (Raytracer.cpp:944-953), unchanged, compiled against
// the drop-in header include/Raytracer.h and linked with lib580rt.so
// (tests/test_dropin.py). Run from a directory that holds Assets/.
#include "Raytracer.h"

int main() {
	//For recording duration stats

	//Do ray tracing
	Raytracer rt(500, 500);
	rt.LoadSceneJSON("simpleSphereScene.json");
	rt.Render("output.ppm");

	return 0;
}
